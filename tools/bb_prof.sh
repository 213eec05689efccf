#!/bin/bash
# Per-kernel backbone breakdown (tools/bb_kernels.py under rocprofv3's kernel
# trace) for each library variant named: bash tools/bb_prof.sh base all ...
# (variants/NAME.so; "main" = the product library).  Each step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in "$@"; do
  lib=variants/$v.so; [ "$v" = main ] && lib=pvnet_amd/libpvvote.so
  PVVOTE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d "$PWD/gpurun_out/bbp_$v" -o bb -- python3 tools/bb_kernels.py > gpurun_out/bbp_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/bbp_$v.log; exit 1; }
  python3 tools/bb_kernels.py --summary gpurun_out/bbp_$v/bb_kernel_trace.csv > gpurun_out/bbp_$v.txt
  rm -f gpurun_out/bbp_$v/bb_kernel_trace.csv
  echo "== $v"; cat gpurun_out/bbp_$v.txt | sed 's/_ZN12_GLOBAL__N_1//' | cut -c1-80
done
