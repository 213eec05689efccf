#!/bin/bash
# rocprof kernel time of k_vote_bytes (tools/u1_probe.py) per variant library
# (VARIANTS="name ..." -> variants/<name>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$PWD/gpurun_out/u1p_$v" -o u1 -- python3 tools/u1_probe.py > gpurun_out/u1p_$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/u1p_{v}/u1_kernel_stats.csv")):
    if "vote_bytes" in r["Name"]:
        print(v, r["Name"][:20], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us avg", round(float(r["MinNs"]) / 1000, 2), "min")
PY
done
