"""Golden fixture G4: the REFERENCE's own ``PVnet``
(lib/networks/model_repository.py:7-79 over lib/networks/resnet.py:116-233),
run in this container on torch-CPU, fp32, with seeded weights.

Container-only (/root/reference does not exist on the GPU box; the tests read
only the .npz this writes).  How the reference is run:
  * ``lib.utils.config`` (imported by resnet.py:1 for a model directory) needs
    ``easydict``, which is absent: a module with a plain ``cfg`` namespace is
    bound under that name instead.  Nothing in the forward reads it.
  * ``PVnet.__init__`` asks for ``resnet18(pretrained=True)`` (MR:13-16), whose
    ``model_zoo.load_url`` (RN:231-232) downloads from the internet.  The
    name ``resnet18`` inside model_repository is rebound to call the
    reference's own ``resnet18`` with pretrained=False, and
    ``model_zoo.load_url`` is replaced by a function that raises, so no
    download can happen.  The random init this skips is overwritten anyway.
  * The seeded state dict (tests/backbone_init.py) is loaded into the
    reference network with ``load_state_dict(strict=True)`` -- the key-set
    and shape equality with ``pvnet_amd.network.PVNet`` -- and the reference's
    eval-mode outputs are recorded on a 1x3x64x80 input and on one 480x640
    frame (a strided lattice, a 32x32 window and per-channel sums of it).
  * Also recorded: how far the reference itself moves in fp16 (CPU half
    convolutions, small input) -- context for the fp16 device tolerance.

Run:  python tests/golden/make_golden_backbone.py  (writes tests/golden/backbone_g4.npz)
"""
from __future__ import annotations

import importlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("PVNET_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from tests import backbone_init as BI  # noqa: E402


def reference_pvnet_module():
    cfg_mod = types.ModuleType("lib.utils.config")
    cfg_mod.cfg = types.SimpleNamespace(MODEL_DIR=os.path.join(REF, "data", "model"))
    sys.modules["lib.utils.config"] = cfg_mod
    import torch.utils.model_zoo as mz

    def _no_download(*a, **k):
        raise RuntimeError("model_zoo.load_url blocked (offline fixture generation)")
    mz.load_url = _no_download
    sys.path.insert(0, REF)
    try:
        rn = importlib.import_module("lib.networks.resnet")
        mr = importlib.import_module("lib.networks.model_repository")
    finally:
        sys.path.remove(REF)
    rn.model_zoo.load_url = _no_download
    mr.resnet18 = lambda pretrained=False, **kw: rn.resnet18(pretrained=False, **kw)
    return mr


def main():
    torch.set_num_threads(8)
    mr = reference_pvnet_module()
    ref = mr.PVnet(18, 2)
    sd = BI.seeded_state_dict(ref.state_dict())
    missing = ref.load_state_dict(sd, strict=True)
    assert not missing.missing_keys and not missing.unexpected_keys
    ref.eval()
    keys = sorted(ref.state_dict())
    shapes = [list(ref.state_dict()[k].shape) for k in keys]
    xs = BI.small_input()
    xf = BI.frame_input()
    with torch.no_grad():
        s_seg, s_ver = ref(torch.from_numpy(xs))
        f_seg, f_ver = ref(torch.from_numpy(xf))
        ref16 = mr.PVnet(18, 2)
        ref16.load_state_dict(sd, strict=True)
        ref16 = ref16.eval().half()
        h_seg, h_ver = ref16(torch.from_numpy(xs).half())
    fs = BI.frame_summary(f_seg.numpy(), f_ver.numpy())
    out = dict(
        seed=np.int64(BI.G4_SEED), weights_sha=BI.weights_sha(sd),
        keys=np.array(keys), shapes=np.array(["x".join(map(str, s)) for s in shapes]),
        x_small=xs, seg_small=s_seg.numpy(), ver_small=s_ver.numpy(),
        f16_cpu_max_dev=np.float64(max(np.abs(h_seg.float().numpy() - s_seg.numpy()).max(),
                                       np.abs(h_ver.float().numpy() - s_ver.numpy()).max())),
        frame_lattice=fs["lattice"], frame_window=fs["window"], frame_chan_sum=fs["chan_sum"],
        frame_input_sha=BI.sha(xf),
    )
    path = os.path.join(HERE, "backbone_g4.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes;", len(keys), "keys; weights", out["weights_sha"][:16])
    print("small out range", float(np.abs(s_seg.numpy()).max()), float(np.abs(s_ver.numpy()).max()),
          "fp16 max dev", float(np.abs(h_ver.float().numpy() - s_ver.numpy()).max()))


if __name__ == "__main__":
    main()
