#!/bin/bash
# full GPU tests + a short bench with every leg
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r04_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04_gpu_tests.log | head; exit $rc; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --skip-cpu > gpurun_out/r04_bench_legs.log 2>&1 || { tail -20 gpurun_out/r04_bench_legs.log; exit 1; }
echo done
