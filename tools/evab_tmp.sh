cd $GRAFT_REPO_ROOT
for rep in 1 2; do for sp in 0 1; do
  TAIL_SPLIT=$sp timeout -k 10 200 python3 tools/bb_kernels.py > gpurun_out/bbsp_$sp.$rep.log 2>&1 || exit 1
  echo "split=$sp $rep $(grep 'ms per forward' gpurun_out/bbsp_$sp.$rep.log)"
done; done
for sp in 0 1; do
  TAIL_SPLIT=$sp timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/ev_$sp -o ev -- python3 tools/e2e_vote_probe.py > gpurun_out/ev_$sp.log 2>&1 || exit 1
  echo "== split=$sp $(grep 'ms per batch' gpurun_out/ev_$sp.log)"
  grep -E '"k_(fg_count|compact|vote_mfma|hyp_gen|refine_solve|decoder_tail)"' gpurun_out/ev_$sp/ev_kernel_stats.csv | cut -d, -f1,4
done
for v in fgnarrow main fgnarrow main; do
  lib=variants/$v.so; [ $v = main ] && lib=pvnet_amd/libpvvote.so
  PVVOTE_LIB=$lib timeout -k 10 200 python3 tools/e2e_vote_probe.py > gpurun_out/evfg_$v.log 2>&1 || exit 1
  echo "== fg $v $(grep 'ms per batch' gpurun_out/evfg_$v.log)"
done
