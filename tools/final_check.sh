# the full GPU suite + smoke, then every single-GPU config line
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_full_tests.sh || exit 3
bash tools/gpu_configs.sh ${1:-final}
