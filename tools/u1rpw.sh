cd $GRAFT_REPO_ROOT
for r in 16; do
  PVVOTE_BYTES_RPW=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/rpw$r -o p -- python3 tools/u1_probe.py > gpurun_out/rpw$r.log 2>&1 || exit 1
done
