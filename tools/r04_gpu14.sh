#!/bin/bash
# decoder tail: branch-free five-row halo build (parity, probe A/B, stamps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_backbone.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t14_tests.log 2>&1 || { tail -30 gpurun_out/t14_tests.log; exit 1; }
tail -1 gpurun_out/t14_tests.log
for rep in 1 2; do
  for v in tail_orig base cur; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 120 python3 tools/tail_probe.py 30 > gpurun_out/t14_tp_$v.$rep.log 2>&1 || exit $?
    echo "$v $rep $(cat gpurun_out/t14_tp_$v.$rep.log | tail -1)"
  done
done
PVVOTE_LIB=variants/tail_trace.so timeout -k 10 120 python3 tools/tail_trace.py > gpurun_out/t14_trace.log 2>&1 || { tail -20 gpurun_out/t14_trace.log; exit 1; }
tail -10 gpurun_out/t14_trace.log
echo done
