set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TRAIN_STEPS=20 TRAIN_WARMUP=3 bash tools/ab_train_env.sh 3 "" A2M_DGRAD_TAP=0 A2M_DGRAD_TAP=1 || exit 3
TRAIN_STEPS=20 TRAIN_WARMUP=3 TRAIN_ARGS="--dtype bf16 --batch 32" bash tools/ab_train_env.sh 2 "" A2M_DGRAD_TAP=0 A2M_DGRAD_TAP=1
