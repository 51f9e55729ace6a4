#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_i2c.log 2>&1 || { tail -30 gpurun_out/pt_i2c.log; exit 4; }
tail -1 gpurun_out/pt_i2c.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_i2c -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/b_i2c.log 2>&1 || { tail -20 gpurun_out/b_i2c.log; exit 5; }
f=$(find gpurun_out/prof_i2c -name '*kernel_stats.csv' | head -1); grep -i "im2col" "$f"
python - <<PY
import csv,collections
rows=[r for r in csv.DictReader(open("gpurun_out/prof_i2c/run_kernel_trace.csv")) if "im2col2d" in r["Kernel_Name"]]
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
d=collections.defaultdict(list)
for i,r in enumerate(rows): d[i%3].append((int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1000)
for k,v in d.items(): v.sort(); print(k,len(v),"median",v[len(v)//2])
PY
