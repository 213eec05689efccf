#!/bin/bash
# round 4 checkpoint B: the driver's bench command plain and under rocprofv3
# (kernel trace + stats, U1/U4 launch summaries, alone/overlapped phases),
# then the backbone's per-kernel trace and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/prof_bench.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_cur" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_cur.log 2>&1 || exit $?
python3 tools/bb_kernels.py --summary gpurun_out/bbk_cur/bb_kernel_trace.csv > gpurun_out/bbk_cur.txt
bash tools/bb_pmc.sh cur || exit $?
echo done
