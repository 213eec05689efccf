#!/bin/bash
# decoder tail: direct blend + LDS-DMA fetch + 3 blocks/CU (parity, probe A/B,
# backbone A/B), then the refine blocks-per-keypoint A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_backbone.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t12_tests.log 2>&1 || { tail -30 gpurun_out/t12_tests.log; exit 1; }
tail -3 gpurun_out/t12_tests.log
for rep in 1 2; do
  for v in tail_orig tail_w2 base tail_w3r14; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 120 python3 tools/tail_probe.py 30 > gpurun_out/t12_tp_$v.$rep.log 2>&1 || exit $?
    echo "$v $rep $(cat gpurun_out/t12_tp_$v.$rep.log | tail -1)"
  done
done
bash tools/bb_ab.sh tail_orig base || exit $?
bash tools/lat_ab.sh nj8 nj16 nj32 || exit $?
echo done
