#!/bin/bash
# k_conv3x3 diagnosis: ablations (no loads / no MFMAs) and SQ counters of the current kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1
for v in cur noloads nomfma; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/bbk_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbk_$v.log 2>&1 || exit $?
  python3 tools/bb_kernels.py --summary gpurun_out/bbk_$v/bb_kernel_trace.csv > gpurun_out/bbk_$v.txt
done
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  PVVOTE_LIB=variants/cur.so timeout -k 10 240 rocprofv3 --kernel-include-regex "k_conv3x3" --pmc $c -T --output-format csv \
    -d "$PWD/gpurun_out/convpmc_$i" -o p -- python3 tools/bb_kernels.py > gpurun_out/convpmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/convpmc_$i.log; }
done
python3 tools/bb_pmc_summary.py gpurun_out/convpmc_1 gpurun_out/convpmc_2 gpurun_out/convpmc_3 gpurun_out/convpmc.json
echo done
