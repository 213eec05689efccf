"""Debug: bench.measure_u1 alone (for comparing its event timing with rocprof's)."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

r = bench.measure_u1(torch.device("cuda"))
print({k: r[k] for k in ("ms", "frac", "traffic")})
