#!/bin/bash
# Round checkpoint: GPU tests, the default bench line (kernel trace kept), every single-GPU config
#   tools/gpu_full.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-full}
bash tools/gpu_check.sh $TAG || exit $?
bash tools/gpu_configs.sh $TAG
