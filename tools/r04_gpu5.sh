#!/bin/bash
# window-form conv: parity, then A/B vs the per-tap form
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PVVOTE_LIB=variants/win.so timeout -k 10 300 python -u -m pytest tests/test_backbone.py -m gpu -x -v -k "conv3x3 or device_fp16 or pvnet42 or inference_form" --timeout 120 --timeout-method thread > gpurun_out/r04_t_win.log 2>&1 || { echo "tests win rc=$?"; grep -E "FAIL|Error|error|max dev" gpurun_out/r04_t_win.log | head -30; exit 1; }
tail -1 gpurun_out/r04_t_win.log
bash tools/bb_ab.sh nowin win || exit $?
for v in win; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
echo done
