"""Build libpvvote.so (the HIP C-ABI library) in-tree for gfx950.

    python -m pvnet_amd.build            # or __graft_entry__.build()

hipcc cross-compiles without a GPU.  The .so lands next to this file so it
travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "pvvote.hip")
SRCS = [SRC, os.path.join(HERE, "csrc", "pvpnp.hip"), os.path.join(HERE, "csrc", "pvdecoder.hip"),
        os.path.join(HERE, "csrc", "pvconv.hip")]
HDR = os.path.join(REPO, "include", "pvvote.h")
OUT = os.path.join(HERE, "libpvvote.so")
ARCH = os.environ.get("PVVOTE_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # every expression restating reference arithmetic rounds after each op;
    # the approximate test's FMAs are explicit fmaf() calls
    "-ffp-contract=off",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    # packed f32 (v_pk_*) has no throughput advantage on gfx950 and costs
    # the abs/neg source modifiers the vote test relies on
    "-fno-slp-vectorize",
    "-fno-gpu-rdc",
    # MFMA results straight into VGPRs (gfx950's unified register file): the
    # vote kernel's VALU reads them without v_accvgpr_read copies
    "-mllvm", "-amdgpu-mfma-vgpr-form=1",
    "-Wall",
]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm install required to build libpvvote.so)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in (*SRCS, HDR, __file__))


def build(force: bool = False, extra=()) -> str:
    if force or needs_build():
        cmd = [hipcc(), *HIPCC_FLAGS, *extra, "-o", OUT + ".tmp", *SRCS]
        subprocess.check_call(cmd)
        # every reference resolved (an unresolved kernel stub only shows at load time)
        import ctypes
        ctypes.CDLL(os.path.abspath(OUT + ".tmp"), mode=ctypes.RTLD_LOCAL | os.RTLD_NOW)
        os.replace(OUT + ".tmp", OUT)
    return OUT


def asm(path: str = os.path.join(HERE, "csrc", "pvvote.gfx950.s")) -> str:
    """Device assembly for inspection (kernel resource usage, v_cmp/s_bcnt1 loops)."""
    cmd = [hipcc(), *[f for f in HIPCC_FLAGS if f not in ("-shared", "-fPIC", "-Wall")],
           "--cuda-device-only", "-S", "-o", path, SRC]
    subprocess.check_call(cmd)
    return path


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
