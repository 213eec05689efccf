#!/bin/bash
# Backbone A/B of library variants (variants/*.so): fp16 batch-32 forward per
# variant, two interleaved rounds on one box, each run time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 200 python3 tools/bb_kernels.py > gpurun_out/bbab_$v.$rep.log 2>&1 || exit $?
    echo "$v $rep $(grep 'ms per forward' gpurun_out/bbab_$v.$rep.log)"
  done
done
