#!/bin/bash
# VALU/SALU instruction counts of k_vote_count for a library variant: tools/ab_pmc.sh <variant>
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
v=$1
PVVOTE_BENCH_NOCHECK=1 PVVOTE_LIB=variants/$v.so timeout -k 10 300 rocprofv3 --kernel-include-regex k_vote_count --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CU_CYCLES -T --output-format csv -d "$PWD/gpurun_out/pmc_$v" -o v -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 10 > gpurun_out/pmc_$v.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_$v
