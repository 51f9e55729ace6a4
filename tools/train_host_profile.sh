# host-side profile of the bf16 B=32 training iteration (cProfile of bench.py --mode train)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -m cProfile -o gpurun_out/train_host.prof bench.py --mode train --steps 10 --warmup 2 --batch 32 --dtype bf16 --no-cpu-baseline > gpurun_out/train_host.log 2>&1 || { tail -5 gpurun_out/train_host.log; exit 3; }
tail -1 gpurun_out/train_host.log
python -c "
import pstats
p = pstats.Stats('gpurun_out/train_host.prof')
p.sort_stats('tottime').print_stats(30)
" > gpurun_out/train_host_tottime.txt
python -c "
import pstats
p = pstats.Stats('gpurun_out/train_host.prof')
p.sort_stats('cumulative').print_stats(40)
" > gpurun_out/train_host_cum.txt
head -60 gpurun_out/train_host_tottime.txt | tail -45
