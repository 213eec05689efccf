"""Deterministic, platform-independent PVNet weights for the backbone parity
fixture G4.  Test infrastructure only.

The reference ships no checkpoint (README.md:101 points to a download), so
G4 pins the *network definition*: the same seeded state dict is loaded into
the reference ``PVnet`` (lib/networks/model_repository.py:7-79, built with
pretrained=False) by ``tests/golden/make_golden_backbone.py`` and into
``pvnet_amd.network.PVNet`` by the tests; both must produce the recorded
outputs.  Weights come from numpy's PCG64 stream (bit-identical on every
platform), so the GPU box regenerates exactly the weights the fixture was
made with; ``weights_sha`` in the fixture checks that.
"""
from __future__ import annotations

import hashlib

import numpy as np
import torch

G4_SEED = 4242


def seeded_state_dict(template: dict, seed: int = G4_SEED) -> dict:
    """A state dict with the keys / shapes / dtypes of `template`, filled
    deterministically: convs He-normal on fan-in, BN affine and running
    statistics randomised (so eval-mode BN is not an identity), biases small."""
    rng = np.random.default_rng(seed)
    out = {}
    for k in sorted(template):
        t = template[k]
        shp = tuple(t.shape)
        if k.endswith("num_batches_tracked"):
            a = np.zeros(shp, np.int64)
        elif k.endswith("running_var"):
            a = rng.uniform(0.6, 1.4, shp).astype(np.float32)
        elif k.endswith("running_mean"):
            a = (rng.standard_normal(shp, dtype=np.float32) * 0.1).astype(np.float32)
        elif len(shp) == 4:
            fan_in = shp[1] * shp[2] * shp[3]
            a = (rng.standard_normal(shp, dtype=np.float32) * np.float32(np.sqrt(2.0 / fan_in))).astype(np.float32)
        elif k.endswith("weight"):          # BN gamma
            a = rng.uniform(0.7, 1.3, shp).astype(np.float32)
        else:                               # BN beta, conv bias
            a = (rng.standard_normal(shp, dtype=np.float32) * 0.05).astype(np.float32)
        out[k] = torch.from_numpy(a)
    return out


def weights_sha(sd: dict) -> str:
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k].detach().cpu().numpy()).tobytes())
    return h.hexdigest()


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def small_input(seed: int = G4_SEED + 1, H: int = 64, W: int = 80) -> np.ndarray:
    return np.random.default_rng(seed).standard_normal((1, 3, H, W), dtype=np.float32)


def frame_input(seed: int = G4_SEED + 2) -> np.ndarray:
    """One ImageNet-normalised-scale 480x640 frame (LINEMOD size)."""
    return np.random.default_rng(seed).standard_normal((1, 3, 480, 640), dtype=np.float32)


# what the fixture keeps of the 480x640 outputs (a full frame is 24.6 MB):
# a 16-px strided lattice and one full 32x32 window per channel
FRAME_STRIDE = 16
FRAME_WIN = (slice(224, 256), slice(304, 336))


def frame_summary(seg: np.ndarray, ver: np.ndarray) -> dict:
    x = np.concatenate([seg, ver], 1)[0]                  # [20, 480, 640]
    return dict(lattice=np.ascontiguousarray(x[:, ::FRAME_STRIDE, ::FRAME_STRIDE]),
                window=np.ascontiguousarray(x[:, FRAME_WIN[0], FRAME_WIN[1]]),
                chan_sum=x.astype(np.float64).sum((1, 2)))


# The mask fixtures (backbone_g4_masks.npz): the seeded weights with the seg
# head's foreground logit shifted so that about half of the random frame is
# foreground -- a mask with long boundaries, i.e. many pixels near the argmax
# decision -- instead of the ~2 % the plain seeded weights give.
SEG_BIAS_KEY = "convraw.3.bias"


def mask_state_dict(template: dict, shift: float, seed: int = G4_SEED) -> dict:
    """seeded_state_dict with ``shift`` subtracted from the foreground logit's
    bias (channel 1 of the last convolution, MR:58 / MR:76)."""
    sd = seeded_state_dict(template, seed)
    b = sd[SEG_BIAS_KEY].clone()
    b[1] = b[1] - np.float32(shift)
    sd[SEG_BIAS_KEY] = b
    return sd


def fg_bits(seg: np.ndarray) -> np.ndarray:
    """torch.argmax(seg_pred, 1) == 1 of a [1, 2, H, W] output (first index on
    ties: class 1 only where l1 > l0), packed (np.packbits, row-major)."""
    return np.packbits((seg[0, 1] > seg[0, 0]).ravel())
