#!/bin/bash
# Round-4 A/B runs that DESIGN.md quotes, one case each (formerly one wrapper
# script per lease): bash tools/r04_runs.sh <case>.  Every GPU step under its
# own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
case "$1" in
gpu15)
# stream throughput against the HIP runtime's hardware queues per process
# (default 4: the 8 in-flight lanes share them pairwise)
INFLIGHT=8 bash tools/ab_env.sh "PVQ=4" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" || exit $?
INFLIGHT=16 bash tools/ab_env.sh "GPU_MAX_HW_QUEUES=16" || exit $?
;;
gpu22)
# (1) halo kernels' multi-tile parity cases; (2) stream images per step (graph granularity) A/B
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
;;
gpu23)
# stream images per step: 512 / 1024 / 2048 (graph granularity), then the full default bench at 1024
for rep in 1 2; do
  for ps in 512 1024 2048; do
    PVVOTE_BENCH_NOCHECK=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --per-step $ps --skip-cpu --skip-e2e --skip-u1 --skip-config3 --skip-u4 > gpurun_out/ps_$ps.$rep.log 2>&1 || exit $?
    python3 - $ps $rep <<'PY'
import json, sys
ps, rep = sys.argv[1:]
d = json.loads([x for x in open(f"gpurun_out/ps_{ps}.{rep}.log") if x.startswith("{")][-1])
print("per_step", ps, rep, "img/s", d["value"], "ms_per_step", d["ms_per_step"], "lat", d["latency_ms_per_image"])
PY
  done
done
/usr/bin/time -v timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --per-step 1024 > gpurun_out/ps_full.log 2> gpurun_out/ps_full.err || { tail -5 gpurun_out/ps_full.err; exit 1; }
grep -E "Elapsed|Maximum resident" gpurun_out/ps_full.err
python3 -c "import json;d=json.loads([x for x in open('gpurun_out/ps_full.log') if x.startswith('{')][-1]);print('full', d['value'], d['roofline']['frac'], d['stream_config3']['images_per_s'], d['stream_config4']['images_per_s'])"
;;
gpu24)
# stream: step graphs in flight (1 = drain between steps, 2 = alternating graphs) A/B; the bench's GPU tests
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
;;
gpu28)
# stream at 1,024 frames per step: frames in flight (lanes) A/B
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
;;
gpu32)
# hypotheses in the vote launch (PVV_HYP_FUSED): the GPU tests, then A/B against k_hyp_gen (latency, stream)
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
;;
gpu37)
# HIP runtime graph-launch knob A/B on the host cost of a 1,024-frame stream replay
for e in "PVQ=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  env $e timeout -k 10 300 python3 tools/replay_host_probe.py 1024 20 > gpurun_out/rh_$e.log 2>&1 || { echo "$e failed rc=$?"; tail -5 "gpurun_out/rh_$e.log"; exit 1; }
  echo "$e"; grep -v amdgpu.ids "gpurun_out/rh_$e.log" | tail -2
done
;;
*) echo "unknown case $1 (gpu15 gpu22 gpu23 gpu24 gpu28 gpu32 gpu37)"; exit 2 ;;
esac
echo done
