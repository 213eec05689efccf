#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_bench_launcher.py -m gpu -x -v -s > gpurun_out/r04_t_launch2.log 2>&1 || { echo "rc=$?"; tail -40 gpurun_out/r04_t_launch2.log; exit 1; }
tail -2 gpurun_out/r04_t_launch2.log
timeout -k 10 300 python -u -m pytest tests/test_backbone.py -m gpu -q -s -k "conv or stem or decoder" > gpurun_out/r04_t_bounds.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r04_t_bounds.log; exit 1; }
grep "vs fp32 conv" gpurun_out/r04_t_bounds.log | head -60
echo done
