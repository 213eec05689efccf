#!/bin/bash
# k_decoder_tail instruction mix / LDS behaviour: PMC passes over
# tools/tail_probe.py (each pass a run of its own).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_decoder_tail" --pmc $C -T --output-format csv \
    -d "$PWD/gpurun_out/tpmc_$i" -o v -- python3 tools/tail_probe.py 5 > gpurun_out/tpmc_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/tpmc_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/tpmc_1 gpurun_out/tpmc_2 2>&1 | tail -40
