#!/bin/bash
# k_conv3x3: s_setprio(1) around the MFMA clusters (A/B on the backbone)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/bb_ab.sh base cv_prio cv_prio0 || exit $?
for v in base cv_prio cv_prio0; do python3 - $v <<'PY'
import sys, re
v = sys.argv[1]
for rep in (1, 2):
    L = open(f"gpurun_out/bbab_{v}.{rep}.log").read().splitlines()
    ks = [l for l in L if "k_conv3x3" in l]
    print(v, rep, " ".join(l.split()[1] for l in ks))
PY
done
echo done
