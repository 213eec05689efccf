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

Run:  python tests/golden/make_golden_backbone.py        (writes tests/golden/backbone_g4.npz)
      python tests/golden/make_golden_backbone.py masks  (writes tests/golden/backbone_g4_masks.npz)
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


def mask_fixture(mr):
    """backbone_g4_masks.npz: the reference's full-frame segmentation masks
    (argmax(seg_pred, 1), tools/demo.py:52, tools/train_linemod.py:254) for
    PVnet(18, 2) and PVnet(42, 2) (configs[4]'s YCB head, MR:8,57), with the
    foreground bias shifted so that half the frame is foreground (the shift
    is computed here from the reference's own output and stored), packed as
    bits; the pixels whose logit margin |l1 - l0| is below 4e-4 of the output
    scale (twice the fp32 device tolerance) with their margins; and for
    PVnet(42, 2) the same small-input outputs / frame summary as G4."""
    xf = torch.from_numpy(BI.frame_input())
    xs = torch.from_numpy(BI.small_input())
    out = {}
    for vd in (18, 42):
        ref = mr.PVnet(vd, 2)
        ref.load_state_dict(BI.seeded_state_dict(ref.state_dict()), strict=True)
        ref.eval()
        with torch.no_grad():
            seg, _ = ref(xf)
        shift = float(np.float32(np.median((seg[0, 1] - seg[0, 0]).numpy())))
        sd = BI.mask_state_dict(ref.state_dict(), shift)
        ref.load_state_dict(sd, strict=True)
        with torch.no_grad():
            seg, ver = ref(xf)
            s_seg, s_ver = ref(xs)
        seg, ver = seg.numpy(), ver.numpy()
        d = (seg[0, 1] - seg[0, 0]).ravel()
        sc = float(np.abs(np.concatenate([seg, ver], 1)).max())
        low = np.nonzero(np.abs(d) < 4e-4 * sc)[0].astype(np.int32)
        out.update({f"shift_{vd}": np.float32(shift), f"weights_sha_{vd}": BI.weights_sha(sd),
                    f"scale_{vd}": np.float64(sc), f"mask_bits_{vd}": BI.fg_bits(seg),
                    f"fg_count_{vd}": np.int64((d > 0).sum()),
                    f"margin_idx_{vd}": low, f"margin_val_{vd}": d[low].astype(np.float32)})
        if vd == 42:
            out.update(seg_small_42=s_seg.numpy(), ver_small_42=s_ver.numpy())
            fs = BI.frame_summary(seg, ver)
            out.update(frame_lattice_42=fs["lattice"], frame_window_42=fs["window"], frame_chan_sum_42=fs["chan_sum"])
        print(f"PVnet({vd}, 2): shift {shift:.4f}, foreground {int((d > 0).sum())} px, scale {sc:.2f}, "
              f"{low.size} px within 4e-4 of scale of the decision")
    out["frame_input_sha"] = BI.sha(BI.frame_input())
    path = os.path.join(HERE, "backbone_g4_masks.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "masks":
        mask_fixture(reference_pvnet_module())
    else:
        main()
