#!/bin/bash
# Build libnewsrec_hip.so into ab/<name>/ with the GEMM translation units (gemm_*.hip) of git
# revision REV and every other object of the in-tree build: a same-box A/B of a GEMM change against
# the revision before it (NR_LIB_PATH).  Run after build().  Usage: tools/build_base_gemm.sh NAME REV
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2
OUT=$ROOT/ab/$NAME
SRC=$(mktemp -d)
mkdir -p $OUT && rm -f $OUT/*.o
(cd $ROOT && git archive $REV news-recommendation-mind_amd/csrc include | tar -x -C $SRC)
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
pids=()
for src in $SRC/news-recommendation-mind_amd/csrc/gemm_*.hip; do
  b=$(basename $src)
  extra=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build; print(' '.join(build.EXTRA.get('$b', [])))")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$SRC/include $extra -c $src -o $OUT/$b.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
objs=$(ls $OBJ/*.o | grep -v "/gemm_[a-z0-9_]*\.hip\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/*.hip.o
rm -rf $SRC
echo $OUT/libnewsrec_hip.so
