#!/bin/bash
# Batch-1 headline stream (tools/stream_timeline.py run) per library variant (variants/*.so), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
for rep in 1 2; do for v in "$@"; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 python -u tools/stream_timeline.py run 10 > gpurun_out/st_$v.$rep.log 2>&1 || exit $?
  echo "$v $rep $(grep '^run:' gpurun_out/st_$v.$rep.log)"
done; done
