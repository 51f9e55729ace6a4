# in-call A/B: the round-2 library (a2m/liba2m_r02.so) against the current one, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
R02=$PWD/audio-to-motion-generation_amd/a2m/liba2m_r02.so
SH="128,32768,4096 64,16384,4096 128,22528,1024 512,4096,2304 256,4096,768 2560,2048,2048"
for v in r02 cur; do
  if [ $v = r02 ]; then export A2M_LIB=$R02; else unset A2M_LIB; fi
  echo "== $v"; timeout -k 10 300 python tools/gemm_bench.py $SH 2>&1 | grep gemm || exit 3
done
for i in 1 2 3; do for v in r02 cur; do
  if [ $v = r02 ]; then export A2M_LIB=$R02; else unset A2M_LIB; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench.json 2>/dev/null || exit 4
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])")"
done; done
