#!/bin/bash
# k_vote_mfma instruction counts (one PMC pass) under profiling-ablation
# builds: VARIANTS="name ..." of variants/<name>.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
for v in $VARIANTS; do
  PVVOTE_LIB=variants/$v.so timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_vote_mfma" --pmc $C -T --output-format csv \
    -d "$PWD/gpurun_out/vmv_$v" -o v -- python3 tools/vote_trace.py > gpurun_out/vmv_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/vmv_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py gpurun_out/vmv_$v | tail -9
done
