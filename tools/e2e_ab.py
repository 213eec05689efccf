"""configs[1] / configs[2] end to end (bench.measure_e2e) under the backbone
forms plain / folded / inference (PVNetInference), interleaved, three rounds.
GPU only."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda:0")
for rep in range(3):
    for half, b, forms in ((True, 32, ("inference", "folded", "plain")), (False, 1, ("inference", "plain", "folded"))):
        for form in forms:
            r = bench.measure_e2e(dev, half=half, batch=b, iters=30, form=form)
            print(f"{rep} {form:9s} {'fp16' if half else 'fp32'} b{b}: {r['images_per_s']:8.1f} img/s, "
                  f"batch {r['ms_per_batch']:.3f} ms, backbone {r['backbone_ms_per_batch']:.3f} ms", flush=True)
