set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/enc_tr -o run -- python tools/enc_trace.py > gpurun_out/enc_tr.log 2>&1 || { tail -5 gpurun_out/enc_tr.log; exit 2; }
cat gpurun_out/enc_tr.log | grep encoder
python - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob('gpurun_out/enc_tr/run_kernel_trace.csv'):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# last 10 graph launches' worth: group by kernel name in order of the final encoder call
seq = rows[-40:]
d = collections.defaultdict(list)
for r in rows[len(rows)//2:]:
    d[r['Kernel_Name'][:70]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f'{k:70s} n={len(v):4d} avg {sum(v)/len(v):7.1f} us')
PY
timeout -k 10 400 python -u tools/tile_probe.py > gpurun_out/r3_probe_m6.txt 2>&1 || { tail -5 gpurun_out/r3_probe_m6.txt; exit 4; }
grep -v "^dense\|MISMATCH" gpurun_out/r3_probe_m6.txt
