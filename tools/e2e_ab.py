"""configs[2] end to end (bench.measure_e2e, fp16 batch 32, PVNetInference),
interleaved A/B of a module-level switch of pvnet_amd.network, three rounds:
    python3 tools/e2e_ab.py [SWITCH]      (default TAIL_SPLIT)
GPU only."""
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import pvnet_amd.network as N  # noqa: E402

sw = sys.argv[1] if len(sys.argv) > 1 else "TAIL_SPLIT"
dev = torch.device("cuda:0")
for rep in range(3):
    for on in (False, True):
        setattr(N, sw, on)
        r = bench.measure_e2e(dev, half=True, batch=32, iters=30)
        print(f"{rep} {sw}={int(on)}: {r['images_per_s']:8.1f} img/s, batch {r['ms_per_batch']:.3f} ms, "
              f"backbone {r['backbone_ms_per_batch']:.3f} ms, voting {r['voting_ms_per_batch']:.3f} ms", flush=True)
