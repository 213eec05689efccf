#!/bin/bash
# conv loop A/B: address precompute (cbm_pre) and loads issued mid-step (cbm_mid) vs cbmajor; parity of both
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in cbm_pre cbm_mid; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_backbone.py -m gpu -x -q -k "conv3x3 or device_fp16 or pvnet42" --timeout 120 --timeout-method thread > gpurun_out/r04_t_$v.log 2>&1 || { echo "tests $v rc=$?"; tail -30 gpurun_out/r04_t_$v.log; exit 1; }
  tail -1 gpurun_out/r04_t_$v.log
done
bash tools/bb_ab.sh cbmajor cbm_pre cbm_mid || exit $?
for v in cbm_pre cbm_mid; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
echo done
