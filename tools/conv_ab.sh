cd "${GRAFT_REPO_ROOT:-/root/repo}"
PVVOTE_LIB=variants/cv_split.so timeout -k 10 200 python -u -m pytest tests/test_backbone.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv3x3" 2>&1 | grep -E "passed|failed"
for r in 1 2; do for v in cv_base cv_split cv_prio cv_splitprio; do
  PVVOTE_LIB=variants/$v.so timeout -k 10 200 python tools/conv_probe.py 1 2>&1 | grep "512->512" | sed "s/^/$v /" || exit 1
done; done
