#!/bin/bash
# tools/pipe_probe.py (bf16 or fp32) under several library builds, one after the other, then the
# per-shape times side by side.   tools/probe_libs.sh "bf16|fp32" "base _ab/x.so _ab/y.so"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PREC=$1; LIBS=$2
ARG=""; [ "$PREC" = bf16 ] && ARG=bf16
files=""
for lib in $LIBS; do
  tag=$(basename $lib .so)
  if [ "$lib" = base ]; then unset A2M_LIB; else export A2M_LIB=$PWD/$lib; fi
  timeout -k 10 150 python tools/pipe_probe.py $ARG > gpurun_out/probe_$tag.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/probe_$tag.log; exit 3; }
  files="$files gpurun_out/probe_$tag.log"
done
unset A2M_LIB
python - $files <<'PY'
import sys, re
cols = []
for f in sys.argv[1:]:
    rows = [l for l in open(f) if ' us ' in l]
    cols.append([(l.split(':')[0].split(' ', 1)[1], float(re.search(r'([\d.]+) us', l).group(1))) for l in rows])
print('shape'.ljust(48) + ''.join(f.split('probe_')[1][:-4].rjust(10) for f in sys.argv[1:]))
for i, (name, _) in enumerate(cols[0]):
    print(name.ljust(48) + ''.join(f'{c[i][1]:10.1f}' for c in cols))
PY
