"""configs[1] / configs[2] end to end (bench.measure_e2e) with BatchNorm folded
vs not, three times each, interleaved.  GPU only."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from pvnet_amd import network  # noqa: E402

fold = network.fold_batchnorm
dev = torch.device("cuda:0")
for rep in range(3):
    for name, f in (("folded", fold), ("bn", lambda n: n)):
        network.fold_batchnorm = f
        for half, b in ((False, 1), (True, 32)):
            r = bench.measure_e2e(dev, half=half, batch=b, iters=30)
            print(f"{rep} {name:6s} {'fp16' if half else 'fp32'} b{b}: {r['images_per_s']:8.1f} img/s, "
                  f"batch {r['ms_per_batch']:.3f} ms, backbone {r['backbone_ms_per_batch']:.3f} ms", flush=True)
