cd $GRAFT_REPO_ROOT
for h in 512 2048; do
  U1_HN=$h timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/hn$h -o p -- python3 tools/u1_probe.py > gpurun_out/hn$h.log 2>&1 || exit 1
done
