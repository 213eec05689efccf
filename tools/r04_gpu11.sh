#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/lat_ab.sh nj8 nj16 nj32 || exit $?
echo done
