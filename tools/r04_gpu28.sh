#!/bin/bash
# stream at 1,024 frames per step: frames in flight (lanes) A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for rep in 1 2; do
  for f in 8 6 12 16; do
    PVVOTE_BENCH_NOCHECK=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --inflight $f --skip-cpu --skip-e2e --skip-u1 --skip-config3 --skip-u4 > gpurun_out/if_$f.$rep.log 2>&1 || exit $?
    python3 - $f $rep <<'PY'
import json, sys
f, rep = sys.argv[1:]
d = json.loads([x for x in open(f"gpurun_out/if_{f}.{rep}.log") if x.startswith("{")][-1])
print("inflight", f, rep, "img/s", d["value"], "ms_per_step", d["ms_per_step"])
PY
  done
done
echo done
