#!/bin/bash
# round 4 final checkpoint on the final code: GPU tests, smoke, the driver's
# bench command plain and under rocprofv3 (stats + U1/U4 summaries + phases),
# then the backbone's per-kernel trace and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04_gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { tail -5 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
bash tools/prof_bench.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_cur" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_cur.log 2>&1 || exit $?
python3 tools/bb_kernels.py --summary gpurun_out/bbk_cur/bb_kernel_trace.csv > gpurun_out/bbk_cur.txt
bash tools/bb_pmc.sh cur || exit $?
echo done
