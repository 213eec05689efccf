cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/ev_w -o ev -- python3 tools/e2e_vote_probe.py > gpurun_out/ev_w.log 2>&1 || exit 1
echo "== $(grep 'ms per batch' gpurun_out/ev_w.log)"
grep -E '"k_(fg_count|compact|compact_wide|vote_mfma|hyp_gen|refine_solve)"' gpurun_out/ev_w/ev_kernel_stats.csv | cut -d, -f1,4
