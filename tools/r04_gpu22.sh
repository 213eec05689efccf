#!/bin/bash
# (1) halo kernels' multi-tile parity cases; (2) stream images per step (graph granularity) A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_backbone.py -q -m gpu -x --timeout 200 --timeout-method thread -k "tail or conv2s or conv4s or conv64" -s > gpurun_out/t22.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/t22.log | head; exit 1; }
grep -E "decoder tail|decoder conv|conv64|passed" gpurun_out/t22.log | tail -24
for rep in 1 2; do
  for ps in ${PSS:-128 256 512}; do
    PVVOTE_BENCH_NOCHECK=1 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --per-step $ps --skip-cpu --skip-e2e --skip-u1 --skip-config3 --skip-u4 > gpurun_out/ps_$ps.$rep.log 2>&1 || exit $?
    python3 - $ps $rep <<'PY'
import json, sys
ps, rep = sys.argv[1:]
d = json.loads([x for x in open(f"gpurun_out/ps_{ps}.{rep}.log") if x.startswith("{")][-1])
print("per_step", ps, rep, "img/s", d["value"], "ms_per_step", d["ms_per_step"])
PY
  done
done
echo done
