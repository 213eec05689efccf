#!/bin/bash
# decoder tail: phase stamps (trace build) + PMC mix of the current form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PVVOTE_LIB=variants/tail_trace.so timeout -k 10 120 python3 tools/tail_trace.py > gpurun_out/t13_trace.log 2>&1 || { tail -20 gpurun_out/t13_trace.log; exit 1; }
cat gpurun_out/t13_trace.log | tail -12
bash tools/tail_pmc.sh || exit $?
echo done
