#!/bin/bash
# Build libnewsrec_hip.so into ab/<name>/ with the working tree's GEMM translation units compiled
# with extra flags (compile-time A/B knobs, e.g. -DNR_AB_MNMN_GUARD=1) and every other object of the
# in-tree build (NR_LIB_PATH selects it).  Run after build().  Usage: tools/build_ab_gemm.sh NAME FLAGS...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/ab/$NAME
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
mkdir -p $OUT && rm -f $OUT/*.o
pids=()
for src in $PKG/csrc/gemm_*.hip; do
  b=$(basename $src)
  extra=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build; print(' '.join(build.EXTRA.get('$b', [])))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include $extra "$@" -c $src -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=$(ls $OBJ/*.o | grep -v "/gemm_[a-z0-9_]*\.hip\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/*.hip.o
echo $OUT/libnewsrec_hip.so
