#!/bin/bash
# k_vote_mfma instruction mix and where its wave cycles go: two PMC passes
# over tools/vote_trace.py's launches (each pass a run of its own).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_vote_mfma" --pmc $C -T --output-format csv \
    -d "$PWD/gpurun_out/vmpmc_$i" -o v -- python3 tools/vote_trace.py > gpurun_out/vmpmc_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 gpurun_out/vmpmc_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/vmpmc_1 gpurun_out/vmpmc_2 2>&1 | tail -30
