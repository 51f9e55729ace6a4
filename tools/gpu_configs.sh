#!/bin/bash
# One bench line per BASELINE config that fits one GPU (configs[1..4]), each under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-cfg}
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/cfg_${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/cfg_${TAG}_$name.log; exit 3; }
  tail -1 gpurun_out/cfg_${TAG}_$name.log > gpurun_out/cfg_${TAG}_$name.json
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms', d['dtype'], d.get('path_roofline',{}).get('frac'))" gpurun_out/cfg_${TAG}_$name.json $name
}
run c2_fp32 --no-cpu-baseline
run c2_bf16 --no-cpu-baseline --dtype bf16
run c5_bf16_b32 --no-cpu-baseline --dtype bf16 --batch 32
run c4_t480_b8 --no-cpu-baseline --frames 480 --batch 8
run c3_train_fp32 --mode train --steps 20 --warmup 5
run c3_train_fp32_b8 --mode train --steps 20 --warmup 5 --batch 8
run c5_train_bf16_b32 --mode train --steps 20 --warmup 5 --batch 32 --dtype bf16
run c3_train_bf16 --mode train --steps 20 --warmup 5 --dtype bf16
exit 0
