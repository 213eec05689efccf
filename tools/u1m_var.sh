#!/bin/bash
# rocprof kernel times of k_vote_bytes_mfma on the U1 probe under
# VARIANTS="name:lib:env ..." (lib "-" = the in-tree library)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for spec in $VARIANTS; do
  IFS=: read -r name lib envs <<< "$spec"
  L=pvnet_amd/libpvvote.so; [ "$lib" != "-" ] && L=variants/$lib.so
  env PVVOTE_LIB=$L ${envs//,/ } timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/u1v_$name" -o u1 -- python3 tools/u1_probe.py > gpurun_out/u1v_$name.log 2>&1 || { tail -20 gpurun_out/u1v_$name.log; exit 1; }
  python3 - $name <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/u1v_{sys.argv[1]}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"]:
        print(f"{sys.argv[1]:12s}", r["Name"][:34], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
done
