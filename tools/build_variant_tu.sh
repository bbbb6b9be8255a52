#!/bin/bash
# Build libnewsrec_hip.so with extra -D flags on ONE translation unit into ab/<name>/ (A/B timing
# against the in-tree build with NR_LIB_PATH).  Run after build().
# Usage: tools/build_variant_tu.sh NAME TU.hip [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; TU=$2; shift 2
OUT=$ROOT/ab/$NAME
mkdir -p $OUT
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include "$@" -c $PKG/csrc/$TU -o $OUT/variant.o
objs=$(ls $OBJ/*.o | grep -v "/$TU\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/variant.o
echo $OUT/libnewsrec_hip.so
