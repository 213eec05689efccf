#!/bin/bash
# round 4, first GPU call: conv parity on the new K order, backbone A/B and PMC traffic of both orders
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
#timeout -k 10 600 python -u -m pytest tests/test_backbone.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_bb_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r04_bb_tests.log; exit 1; }
#tail -3 gpurun_out/r04_bb_tests.log
bash tools/bb_ab.sh tapmajor cbmajor || exit $?
PVVOTE_LIB=variants/tapmajor.so bash tools/bb_pmc.sh tapmajor || exit $?
PVVOTE_LIB=variants/cbmajor.so bash tools/bb_pmc.sh cbmajor || exit $?
for v in tapmajor cbmajor; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --skip-e2e --skip-config3 --skip-cpu > gpurun_out/r04_bench_quick.log 2>&1 || exit $?
echo done
