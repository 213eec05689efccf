"""Wall time of MIOpen's Find and the resulting inference-form forward (fp16
batch 32, f32 batch 1) under the MIOPEN_FIND_MODE of the environment.  GPU only."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda:0")
for half, b in ((True, 32), (False, 1)):
    t0 = time.time()
    r = bench.measure_e2e(dev, half=half, batch=b, iters=30)
    print(f"FIND_MODE={os.environ.get('MIOPEN_FIND_MODE', 'default')} {'fp16' if half else 'fp32'} b{b}: "
          f"{r['images_per_s']:8.1f} img/s, backbone {r['backbone_ms_per_batch']:.3f} ms, wall {time.time() - t0:.1f} s",
          flush=True)
