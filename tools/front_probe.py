"""k_front's hand-off on the device (a diagnostic, GPU only): eager v3 calls on
S(1234) with a PVV_FRONT_STATS build (PVVOTE_LIB=variants/fstats.so), the
flag statistics per call (flags worked out by the waiter, spin rounds, the
longest wait), the time per call, and a batch of 5 against its single calls
(tn, hypotheses, counts per image).

    PVVOTE_LIB=variants/fstats.so python tools/front_probe.py
"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from pvnet_amd import _lib, ransac_voting_gpu as rvg, synth  # noqa: E402


def main():
    L = _lib.load()
    L.pv_debug_front_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    L.pv_debug_front_stats.restype = ctypes.c_int
    st = (ctypes.c_uint64 * 4)()

    def stats():
        torch.cuda.synchronize()
        rc = L.pv_debug_front_stats(st)
        return list(st) if rc == 0 else None

    dev = torch.device("cuda:0")
    fd = synth.synthetic_field(1234)
    seg = torch.from_numpy(fd["seg"]).to(dev)
    ver = torch.from_numpy(fd["vertex"]).to(dev)
    ws = rvg.VotingWorkspace()
    out = torch.zeros((1, 9, 2), device=dev)
    for i in range(3):
        rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _seed=7 + i, _workspace=ws, out=out)
    print("warm stats", stats(), flush=True)
    for i in range(6):
        torch.cuda.synchronize()
        t = time.perf_counter()
        rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _seed=11 + i, _workspace=ws, out=out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) * 1e6
        err = float(np.abs(out.cpu().numpy()[0] - fd["keypoints"]).max())
        print(f"call {i}: {dt:.1f} us, kp err {err:.3f}, stats {stats()}", flush=True)

    b, hn = 5, 128
    fb = synth.synthetic_batch(b, seed=300)
    mask = np.argmax(fb["seg"], 1).astype(np.int64)
    mask[3] = 0
    mask[3, 100:105, 200:210] = 1
    mask[4] = 0
    vertex = np.ascontiguousarray(fb["vertex"].transpose(0, 2, 3, 1).reshape(b, 480, 640, 9, 2))
    rng = np.random.default_rng(31)
    fg = [int((mask[i] != 0).sum()) for i in range(b)]
    idxs = np.stack([rng.integers(0, max(n, 1), (hn, 9, 2)) for n in fg]).astype(np.int32)
    md, vd = torch.from_numpy(mask).to(dev), torch.from_numpy(vertex).to(dev)
    diag = {}
    kb = rvg.ransac_voting_layer_v3(md, vd, hn, _idxs=idxs, _diag=diag).cpu().numpy()
    print("batch stats", stats(), "tn", diag["tn"].cpu().numpy().tolist(), flush=True)
    for i in range(b):
        d1 = {}
        k1 = rvg.ransac_voting_layer_v3(md[i:i + 1], vd[i:i + 1], hn, _idxs=idxs[i:i + 1], _diag=d1).cpu().numpy()
        hb, h1 = diag["hyp"][i].cpu().numpy(), d1["hyp"][0].cpu().numpy()
        cb, c1 = diag["counts"][i].cpu().numpy(), d1["counts"][0].cpu().numpy()
        print(f"image {i}: tn {int(diag['tn'][i])} / {int(d1['tn'][0])}, hyp equal {np.array_equal(hb, h1)} "
              f"({int((hb != h1).any(-1).sum())} differ), counts equal {np.array_equal(cb, c1)}, "
              f"kp max diff {float(np.abs(kb[i] - k1[0]).max()):.4f}, stats {stats()}", flush=True)


if __name__ == "__main__":
    main()
