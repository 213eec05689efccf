"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports
every symbol include/pvvote.h declares, and its host-only entry points work.
Also the host logic of the Python layers that runs before any device call."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(REPO, "include", "pvvote.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pv_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from pvnet_amd import build, _lib
    build.build()
    return _lib.load()


def test_header_symbols_exported(lib):
    names = declared_functions()
    assert len(names) >= 12
    from pvnet_amd import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    for n in names:
        assert hasattr(lib, n), f"{n} declared in pvvote.h but not exported"
        assert n in bound, f"{n} has no ctypes signature in pvnet_amd/_lib.py"


def test_library_is_built_for_gfx950():
    path = os.path.join(REPO, "pvnet_amd", "libpvvote.so")
    blob = open(path, "rb").read()
    assert b"gfx950" in blob


def test_version_and_errors(lib):
    assert lib.pv_version().decode().startswith("pvvote")
    assert lib.pv_error_string(0) == b"ok"
    assert b"invalid" in lib.pv_error_string(-1)
    assert b"workspace" in lib.pv_error_string(-2)


def test_workspace_size_host_only(lib):
    n1 = lib.pv_v3_workspace_size(1, 480, 640, 9, 512)
    n4 = lib.pv_v3_workspace_size(4, 480, 640, 9, 512)
    assert n1 > 480 * 640 * 9 * 8 and n4 > 3 * n1
    assert lib.pv_v3_workspace_size(0, 480, 640, 9, 512) == 0


def test_argument_errors_without_device(lib):
    # invalid arguments are rejected before anything is launched
    assert lib.pv_generate_hypothesis(None, None, None, None, 10, 9, 4, None) == -1
    assert lib.pv_voting_for_hypothesis(None, None, None, None, 10, 9, 4, 0.99, 0, None) == -1
    assert lib.pv_ransac_voting_v3(None, None, None, None, 0, None, None) == -1
    from pvnet_amd import _lib
    d = _lib.ImageDesc(mask=1, vertex=1, b=1, H=4, W=4, vn=9, mask_kind=7)
    p = _lib.VoteParams(round_hyp_num=8)
    assert lib.pv_ransac_voting_v3(ctypes.byref(d), ctypes.byref(p), 1, None, 0, None, None) == -1
    d.mask_kind = 0
    assert lib.pv_ransac_voting_v3(ctypes.byref(d), ctypes.byref(p), 1, None, 0, None, None) == -2


def test_python_layer_rejects_host_tensors():
    from pvnet_amd import ransac_voting as rv
    from pvnet_amd import ransac_voting_gpu as rvg
    d = torch.zeros(10, 3, 2)
    c = torch.zeros(10, 2)
    i = torch.zeros(4, 3, 2, dtype=torch.int32)
    with pytest.raises(RuntimeError, match="CUDA"):
        rv.generate_hypothesis(d, c, i)
    with pytest.raises(RuntimeError, match="CUDA"):
        rvg.ransac_voting_layer_v3(torch.zeros(1, 4, 4, dtype=torch.int64), torch.zeros(1, 4, 4, 3, 2), 8)


def test_b_inv_semantics_host():
    from pvnet_amd.ransac_voting_gpu import b_inv
    A = torch.tensor([[[2., 1.], [1., 3.]], [[4., 0.], [0., 5.]]])
    np.testing.assert_allclose(b_inv(A).numpy(), np.linalg.inv(A.numpy()), rtol=1e-6)
    A[1] = 0
    np.testing.assert_array_equal(b_inv(A).numpy(), np.broadcast_to(np.eye(2), (2, 2, 2)))


def test_synthetic_generator():
    from pvnet_amd import synth
    f = synth.synthetic_field(1234)
    assert f["tn"] == 29861 and f["seg"].shape == (1, 2, 480, 640) and f["vertex"].shape == (1, 18, 480, 640)
    assert (np.argmax(f["seg"][0], 0) == 1).sum() == 29861
    n = np.sqrt(f["vertex"][0, 0::2] ** 2 + f["vertex"][0, 1::2] ** 2)
    assert np.allclose(n[:, f["mask"]], 1.0, atol=1e-6) and np.all(n[:, ~f["mask"]] == 0)
