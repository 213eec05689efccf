#!/bin/bash
# MFMA vote kernel: per-wave traces under several round weights (PVVOTE_VM_RW)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in ${WEIGHTS:-0,0,0,0}; do
  PVVOTE_VM_RW=$w timeout -k 10 120 python tools/vote_trace.py > gpurun_out/vtw_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/vtw_$w.log; exit 1; }
  echo "== $w: $(sed -n 2,2p gpurun_out/vtw_$w.log) | $(grep -E 'per-SIMD last end' gpurun_out/vtw_$w.log) | $(grep 'by start rank' gpurun_out/vtw_$w.log) | $(grep 'fix steps' gpurun_out/vtw_$w.log)"
done
