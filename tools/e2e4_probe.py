"""configs[4] end to end (bench.measure_e2e_config4: PVnet(42, 2) fp16 batch 32
+ v3 + EVD with mean + uncertainty PnP, one graph) for a rocprofv3 kernel
trace: `rocprofv3 --kernel-trace --stats -d DIR -o e4 -- python3 tools/e2e4_probe.py`.
GPU only."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

r = bench.measure_e2e_config4(torch.device("cuda:0"), iters=10)
print(r["images_per_s"], "images/s,", r["ms_per_batch"], "ms per batch")
