#!/bin/bash
# hypotheses in the vote launch (PVV_HYP_FUSED): the GPU tests, then A/B against k_hyp_gen (latency, stream)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t32.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/t32.log | head -20; tail -5 gpurun_out/t32.log; exit 1; }
tail -1 gpurun_out/t32.log
for rep in 1 2; do
  for v in nofuse fused; do
    PVVOTE_LIB=variants/$v.so timeout -k 10 120 python3 tools/lat_trace.py 20 > gpurun_out/l32_$v.$rep.log 2>&1 || exit $?
    PVVOTE_LIB=variants/$v.so PVVOTE_BENCH_NOCHECK=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --skip-cpu --skip-e2e --skip-u1 --skip-u4 > gpurun_out/b32_$v.$rep.log 2>&1 || exit $?
    python3 - $v $rep <<'PY'
import json, sys
v, rep = sys.argv[1:]
lat = [x for x in open(f"gpurun_out/l32_{v}.{rep}.log") if x.startswith("latency")][-1].split()[-1]
d = json.loads([x for x in open(f"gpurun_out/b32_{v}.{rep}.log") if x.startswith("{")][-1])
print(v, rep, "seq_lat_us", lat, "img/s", d["value"], "c3", d["stream_config3"]["images_per_s"], "c4", d["stream_config4"]["images_per_s"],
      "vote_us", round(d["roofline_vote_count"]["avg_kernel_ms"] * 1000, 2), "order_ok", d["stream_order_ok"], d["library"]["build"][-60:])
PY
  done
done
echo done
