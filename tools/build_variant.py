"""Build an A/B variant of libpvvote.so under variants/NAME.so with extra
hipcc defines:  python tools/build_variant.py NAME [-DMACRO=V ...] [--src=pvvote.hip:OLD.hip]
(select it at run time with PVVOTE_LIB=variants/NAME.so).  Not part of the product."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pvnet_amd import build as B  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
srcs = list(B.SRCS)
# --src=NAME.hip:ALT.hip builds with ALT in place of csrc/NAME.hip (e.g. a saved older version)
for e in [e for e in extra if e.startswith("--src=")]:
    k, alt = e[len("--src="):].split(":")
    srcs = [alt if os.path.basename(p) == k else p for p in srcs]
    extra.remove(e)
os.makedirs(os.path.join(B.REPO, "variants"), exist_ok=True)
out = os.path.join(B.REPO, "variants", name + ".so")
subprocess.check_call([B.hipcc(), *B.HIPCC_FLAGS, *extra, "-o", out, *srcs])
print(out)
