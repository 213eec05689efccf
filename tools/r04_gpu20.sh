#!/bin/bash
# k_vote_mfma: hot-loop issue priority by the share left (A/B: latency, stream, vote alone; wave stamps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/lat_ab.sh base vprio || exit $?
PVVOTE_LIB=variants/vprio_tr.so timeout -k 10 200 python3 tools/vote_trace.py > gpurun_out/vtrace_prio.log 2>&1 || exit 1
grep -E "^(end|life|per-SIMD|end after|phase)" gpurun_out/vtrace_prio.log
echo done
