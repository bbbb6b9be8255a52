#!/bin/bash
# Build libnewsrec_hip.so with extra -D flags on gemm_fast.hip into ab/<name>/ (A/B timing with
# NR_LIB_PATH).  Usage: tools/build_variant.sh NAME [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/ab/$NAME
mkdir -p $OUT
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include "$@" -c $PKG/csrc/gemm_fast.hip -o $OUT/gemm_fast.o
objs=$(ls $OBJ/*.o | grep -v "/gemm_fast.hip\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/gemm_fast.o
echo $OUT/libnewsrec_hip.so
