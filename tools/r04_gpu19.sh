#!/bin/bash
# k_conv3x3 (256-cout tiles): where the next step's load pieces are issued (A/B on the backbone)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/bb_ab.sh base cv_is3 cv_is4 || exit $?
echo done
