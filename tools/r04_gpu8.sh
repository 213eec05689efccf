#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/ab_libs.sh vlean vlean_bpc1 vlean_bpc2 || exit $?
for v in base base_nomfma win win_nomfma; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
for v in base win; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 240 rocprofv3 --kernel-include-regex "k_conv3x3" --pmc SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE -T --output-format csv \
    -d "$PWD/gpurun_out/convta_$v" -o p -- python3 tools/bb_kernels.py > gpurun_out/convta_$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/convta_$v.log; }
  python3 tools/bb_pmc_summary.py gpurun_out/convta_$v gpurun_out/convta_$v.json | grep 1228800
done
echo done
