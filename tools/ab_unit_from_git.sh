#!/bin/bash
# Build libnewsrec_hip.so into ab/<name>/ with ONE translation unit taken from a git revision (the
# rest from the in-tree build's objects): a same-box A/B of a kernel change.  Run after build().
# Usage: tools/ab_unit_from_git.sh NAME REV UNIT.hip   (e.g. bert_old HEAD bert.hip)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; UNIT=$3
OUT=$ROOT/ab/$NAME
PKG=$ROOT/news-recommendation-mind_amd
OBJ=$PKG/newsrec_amd/lib/obj
mkdir -p $OUT && rm -f $OUT/*.o
git -C $ROOT show $REV:news-recommendation-mind_amd/csrc/$UNIT > $PKG/csrc/.ab_$UNIT
extra=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build; print(' '.join(build.EXTRA.get('$UNIT', [])))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I$ROOT/include $extra -x hip -c $PKG/csrc/.ab_$UNIT -o $OUT/$UNIT.o
rm -f $PKG/csrc/.ab_$UNIT
objs=$(ls $OBJ/*.o | grep -v "/$UNIT\.")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnewsrec_hip.so $objs $OUT/$UNIT.o
echo $OUT/libnewsrec_hip.so
