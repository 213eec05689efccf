#!/bin/bash
# stream: step graphs in flight (1 = drain between steps, 2 = alternating graphs) A/B; the bench's GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_bench_launcher.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/t24.log 2>&1 || { tail -20 gpurun_out/t24.log; exit 1; }
tail -1 gpurun_out/t24.log
for rep in 1 2; do
  for sg in 1 2 3; do
    PVVOTE_BENCH_NOCHECK=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --step-graphs $sg --skip-cpu --skip-e2e --skip-u1 --skip-u4 > gpurun_out/sg_$sg.$rep.log 2>&1 || exit $?
    python3 - $sg $rep <<'PY'
import json, sys
sg, rep = sys.argv[1:]
d = json.loads([x for x in open(f"gpurun_out/sg_{sg}.{rep}.log") if x.startswith("{")][-1])
print("step_graphs", sg, rep, "img/s", d["value"], "ms_per_step", d["ms_per_step"], "lat", d["latency_ms_per_image"],
      "order_ok", d["stream_order_ok"], "kp_err", d["max_kp_err_px"], "c3", d["stream_config3"]["images_per_s"], "c4", d["stream_config4"]["images_per_s"])
PY
  done
done
echo done
