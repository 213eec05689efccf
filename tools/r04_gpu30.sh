#!/bin/bash
# diagnostic: a deep stream graph (4,096 frames: 2,560 dependent kernels per lane);
# STACK_KB set: under that stack limit
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
if [ -n "$STACK_KB" ]; then ulimit -s "$STACK_KB" || exit 3; fi
echo "stack limit: $(ulimit -s) (hard $(ulimit -Hs))"
timeout -k 10 300 python3 -X faulthandler tools/deep_graph_probe.py 4096 > gpurun_out/dg_${STACK_KB:-default}.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "per_step|File|Fatal" gpurun_out/dg_${STACK_KB:-default}.log | head -8
exit $rc
