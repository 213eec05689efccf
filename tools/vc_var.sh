#!/bin/bash
# vote kernel variants (variants/<name>.so built with ablation macros):
# per-wave trace summary of each
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 120 python tools/vote_trace.py > gpurun_out/vt_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/vt_$v.log; exit 1; }
  echo "== $v: $(sed -n 2,2p gpurun_out/vt_$v.log) $(grep -E 'first hot loop' gpurun_out/vt_$v.log)"
  grep -E "^end |slow sub|fix steps|per-SIMD last end|by start rank" gpurun_out/vt_$v.log
done
