#!/bin/bash
# vote kernel: registers 155 -> 124, LDS 44 -> 39 KiB; correctness then stream A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vote_mfma.py tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_vote_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error" gpurun_out/r04_vote_tests.log | head; exit 1; }
tail -1 gpurun_out/r04_vote_tests.log
bash tools/ab_libs.sh vbase vlean384 vlean vlean_bpc4 || exit $?
echo done
