#!/bin/bash
# stream images per step: 512 / 1024 / 2048 (graph granularity), then the full default bench at 1024
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
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
echo done
