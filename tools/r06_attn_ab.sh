#!/bin/bash
# Fused eval attention with 128-channel V chunks (in-tree) vs 64-channel chunks (_ab/nv64.so):
# the attention / grouped / bf16 / headline tests, then interleaved bench lines and one replayed-step
# breakdown each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grouped.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread -k "attention or headline or grouped or bf16" > gpurun_out/at_pytest.log 2>&1 || { tail -30 gpurun_out/at_pytest.log; exit 1; }
tail -1 gpurun_out/at_pytest.log
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/nv64.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/at_b.log 2>&1 || { echo "bench $lib failed"; tail -5 gpurun_out/at_b.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/at_b16.log 2>&1 || { echo "bench bf16 $lib failed"; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/at_b.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 $(python -c "import json; print(json.loads(open('gpurun_out/at_b16.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
export TMPDIR=/tmp
for lib in $L0 $PWD/_ab/nv64.so; do
  n=$(basename $lib .so)
  A2M_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/at_tr_$n -o run -- python tools/step_pmc.py 10 --sync --engine-json gpurun_out/at_eng_$n.json > gpurun_out/at_tr_$n.log 2>&1 || { echo "trace $n failed"; tail -5 gpurun_out/at_tr_$n.log; exit 4; }
  GF=$(python -c "import json; print(json.load(open('gpurun_out/at_eng_$n.json'))['gflop'])")
  python tools/replay_breakdown.py gpurun_out/at_tr_$n 10 --gflop $GF --out gpurun_out/at_breakdown_$n.txt > /dev/null || exit 5
  python tools/step_lanes.py gpurun_out/at_tr_$n 3 > gpurun_out/at_lanes_$n.txt || exit 6
  echo $n; grep -E "span|attn" gpurun_out/at_breakdown_$n.txt
  find gpurun_out/at_tr_$n -name "*kernel_trace.csv" -delete
done
exit 0
