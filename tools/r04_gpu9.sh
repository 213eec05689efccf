#!/bin/bash
# conv: 8-wave blocks (128 x 64 per wave) with / without the step's fragments read ahead
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PVVOTE_LIB=variants/nw8fa.so timeout -k 10 300 python -u -m pytest tests/test_backbone.py -m gpu -x -q -k "conv3x3" --timeout 120 --timeout-method thread > gpurun_out/r04_t_nw8fa.log 2>&1 || { echo "tests rc=$?"; grep -E "FAILED|Error|error" gpurun_out/r04_t_nw8fa.log | head; exit 1; }
tail -1 gpurun_out/r04_t_nw8fa.log
bash tools/bb_ab.sh base nw8 nw8fa || exit $?
for v in base nw8 nw8fa; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
echo done
