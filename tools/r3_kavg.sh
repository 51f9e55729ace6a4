# per-kernel average durations of the bench step for the in-tree and the prev library
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PAT=${1:-attn_fused_eval}
for v in new prev new prev; do
if [ $v = prev ]; then export A2M_LIB=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so; else unset A2M_LIB; fi
rm -rf gpurun_out/kavg
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/kavg -o run -- python tools/step_pmc.py 10 > gpurun_out/kavg.log 2>&1 || { tail -5 gpurun_out/kavg.log; exit 3; }
echo "$v: $(python tools/prof_summary.py gpurun_out/kavg/run_kernel_trace.csv 12 | grep -E "$PAT" | head -3 | tr -s ' ' | tr '\n' '|')"
done
