#!/bin/bash
# Build libnewsrec_hip.so with extra flags on the GEMM translation units (gemm_*.hip; every unit
# with ALL=1) into ab/<name>/ (A/B timing with NR_LIB_PATH).  Usage: [ALL=1] tools/build_variant.sh NAME [-DFLAG ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OUT=$ROOT/ab/$NAME
mkdir -p $OUT && rm -f $OUT/*.o
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
pids=()
PAT="gemm_*.hip"
[ "${ALL:-0}" = 1 ] && PAT="*.hip"
for src in $PKG/csrc/$PAT; do
  b=$(basename $src)
  extra=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build; print(' '.join(build.EXTRA.get('$b', [])))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include $extra "$@" -c $src -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
if [ "${ALL:-0}" = 1 ]; then
  objs="$OBJ/version.o"
else
  objs=$(ls $OBJ/*.o | grep -v "/gemm_[a-z0-9_]*\.hip\.")
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/*.hip.o
echo $OUT/libnewsrec_hip.so
