#!/bin/bash
# Diagnostic library variants: the in-tree objects with ONE translation unit rebuilt under extra
# flags, linked into _ab/<name>.so (A2M_LIB=_ab/<name>.so selects it at run time).
#   tools/build_variant.sh NAME TU "FLAGS"     e.g.  tools/build_variant.sh abl1 gemm_f32_pipe "-DA2M_PIPE_ABL=1"
set -eu
cd "$(dirname "$0")/../audio-to-motion-generation_amd"
NAME=$1; TU=$2; FLAGS=$3
mkdir -p ../_ab /tmp/a2m_var_$NAME
HIPFLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics -ffp-contract=fast"
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c csrc/$TU.hip -o /tmp/a2m_var_$NAME/$TU.o
OBJS=$(ls build/*.o | grep -v "/$TU.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS /tmp/a2m_var_$NAME/$TU.o -o ../_ab/$NAME.so
echo "built _ab/$NAME.so"
