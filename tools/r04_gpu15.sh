#!/bin/bash
# stream throughput against the HIP runtime's hardware queues per process
# (default 4: the 8 in-flight lanes share them pairwise)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
INFLIGHT=8 bash tools/ab_env.sh "PVQ=4" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" || exit $?
INFLIGHT=16 bash tools/ab_env.sh "GPU_MAX_HW_QUEUES=16" || exit $?
echo done
