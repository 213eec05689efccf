#!/bin/bash
# Instruction mix of the vote kernels (new MFMA kernel and the VALU one):
# one PMC pass each over tools/vote_trace.py's four launches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY"
for v in new old; do
  e=""; [ $v = old ] && e="PVVOTE_VC_OLD=1"
  env $e timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_vote_(mfma|count)" --pmc $C -T --output-format csv \
    -d "$PWD/gpurun_out/vcpmc_$v" -o v -- python3 tools/vote_trace.py > gpurun_out/vcpmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/vcpmc_$v.log; exit 1; }
done
echo ok
