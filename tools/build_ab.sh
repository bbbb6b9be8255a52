#!/bin/bash
# Build libnewsrec_hip.so into ab/<name>/ with some of the working tree's translation units compiled
# with extra flags (compile-time A/B knobs) and every other object of the in-tree build (NR_LIB_PATH
# selects it).  Run after build().  Usage: [AB_SRCS=glob AB_RE=regex] tools/build_ab.sh NAME FLAGS...
# (default: the GEMM units, gemm_*.hip / gemm_[a-z0-9_]*; e.g. AB_SRCS=score_adam.hip AB_RE=score_adam)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/ab/$NAME
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
mkdir -p $OUT && rm -f $OUT/*.o
pids=()
for src in $(ls $PKG/csrc/${AB_SRCS:-gemm_*.hip}); do
  b=$(basename $src)
  extra=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build; print(' '.join(build.EXTRA.get('$b', [])))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include $extra "$@" -c $src -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=$(ls $OBJ/*.o | grep -v -E "/(${AB_RE:-gemm_[a-z0-9_]*})\.hip\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/*.hip.o
echo $OUT/libnewsrec_hip.so
