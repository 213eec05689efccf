#!/bin/bash
# Stream throughput against images in flight and the vote kernel's blocks per
# CU (PVVOTE_VM_BPC); two interleaved rounds, each run time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in ${CFGS:-"8 3" "6 3" "12 3" "16 3" "8 2" "12 2"}; do
    set -- $cfg
    PVVOTE_BENCH_NOCHECK=1 PVVOTE_VM_BPC=$2 timeout -k 10 200 python bench.py --inflight $1 --steps 50 --warmup 10 \
      --skip-cpu --skip-e2e --skip-u1 > gpurun_out/ifab_$1_$2.$rep.log 2>&1 || exit $?
    python - "$1" "$2" "$rep" <<'PY'
import json, sys
f, b, rep = sys.argv[1:]
d = json.loads([x for x in open(f"gpurun_out/ifab_{f}_{b}.{rep}.log") if x.startswith("{")][-1])
print("inflight", f, "bpc", b, rep, "img/s", d["value"], "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2))
PY
  done
done
