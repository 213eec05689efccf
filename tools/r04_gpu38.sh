#!/bin/bash
# k_conv3x3 256-cout tiles: the next step's weight pieces before the MFMAs, pixel pieces after the first half (A/B, 3 rounds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in base cv_is3; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 200 python3 tools/bb_kernels.py > gpurun_out/bb38_$v.$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep 'ms per forward' gpurun_out/bb38_$v.$rep.log)"
  done
done
echo done
