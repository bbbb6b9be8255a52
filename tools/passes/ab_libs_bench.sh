# Same-box A/B of library builds on the NRMS bench line: the in-tree build and ab/<name>/ builds
# alternating (rounds), each variant's parity tests first (NR_LIB_PATH), then each variant's step trace.
# Usage: bash tools/passes/ab_libs_bench.sh OUT "name1 name2" "TESTS" [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; mkdir -p $O
VARS=$2; T=$3; R=${4:-3}
echo tests base; timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_base.log 2>&1 || exit 1
for v in $VARS; do
  echo tests $v; NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1 || exit 1
done
B="python bench.py --steps 30 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in $(seq 1 $R); do
  echo round $i
  timeout -k 10 200 $B > $O/bench_base_$i.json 2>> $O/bench.err || exit 3
  for v in $VARS; do
    NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_${v}_$i.json 2>> $O/bench.err || exit 3
  done
done
for v in $VARS; do
  echo trace $v; NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- $B > $O/kt_$v.log 2>&1 || exit 6
done
echo trace base; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_base -o run -- $B > $O/kt_base.log 2>&1 || exit 6
echo done
