#!/bin/bash
# k_vote_count instruction counts per variant library (profiling ablations):
# VARIANTS="name ..." -> variants/<name>.so; one --pmc pass per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in $VARIANTS; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 300 rocprofv3 --kernel-include-regex k_vote_count \
    --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    -T --output-format csv -d "$PWD/gpurun_out/vcpmc_$v" -o v -- python3 bench.py --skip-cpu --skip-e2e --skip-u1 --steps 10 \
    > gpurun_out/vcpmc_$v.log 2>&1 || { echo "failed: $v"; tail -5 gpurun_out/vcpmc_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import collections, csv, glob, sys
v = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/vcpmc_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(v, {k: round(sum(x) / len(x) / 1e6, 3) for k, x in sorted(acc.items())}, "(M per dispatch)")
PY
done
