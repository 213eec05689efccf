"""U4 (estimate_voting_distribution_with_mean on S(1234), 16 x 256
hypotheses) alone, for PMC passes: `rocprofv3 --pmc ... -- python3
tools/u4_probe.py [reps]`.  GPU only; not part of the product or the tests."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
r = bench.measure_u4(torch.device("cuda", 0), reps=reps)
print({k: r[k] for k in ("avg_kernel_ms", "reduce_ms", "call_ms", "frac")})
