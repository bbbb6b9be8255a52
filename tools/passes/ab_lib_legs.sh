# Same-box A/B of the in-tree library against ab/base/libnewsrec_hip.so on the configuration legs:
# GEMM shapes (tools/gemm_ab.py), then the legs alternating new / base (tools/legs_only.py), then the
# new build's leg trace.  Usage: bash tools/passes/ab_lib_legs.sh NAME CASES LEGS [TESTS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; mkdir -p $O
CASES=$2; LEGS=$3; T=$4
if [ -n "$T" ]; then
  echo tests; timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/base/libnewsrec_hip.so,base,ab/base/libnewsrec_hip.so --cases $CASES > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
for i in 1 2 3; do
  echo round $i
  timeout -k 10 300 python tools/legs_only.py $LEGS --steps 20 > $O/legs_new_$i.json 2>> $O/legs.err || exit 3
  NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/base/libnewsrec_hip.so timeout -k 10 300 python tools/legs_only.py $LEGS --steps 20 > $O/legs_old_$i.json 2>> $O/legs.err || exit 3
done
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/legs_only.py $LEGS --steps 5 > $O/kt.log 2>&1 || exit 6
echo done
