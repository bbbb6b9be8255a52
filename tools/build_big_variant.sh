#!/bin/bash
# Build libnewsrec_hip.so with extra -D flags on the bf16x6 big-tile GEMM translation unit into
# ab/<name>/ (A/B timing against the in-tree build with NR_LIB_PATH).  Run after build().
# Usage: tools/build_big_variant.sh NAME [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/ab/$NAME
mkdir -p $OUT
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include "$@" -c $PKG/csrc/gemm_big_3_256.hip -o $OUT/gemm_big_3_256.o
objs=$(ls $OBJ/*.o | grep -v gemm_big_3_256.hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/gemm_big_3_256.o
echo $OUT/libnewsrec_hip.so
