cd $GRAFT_REPO_ROOT
for d in 0 3; do
  PVVOTE_DEBUG_BYTES=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/u1dbg$d -o p -- python3 tools/u1_probe.py > gpurun_out/u1dbg$d.log 2>&1 || exit 1
done
