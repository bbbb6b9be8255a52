# Same-box A/B of the working tree against ab/base_tree (the Python side of a git revision, `git archive`
# into ab/base_tree) with ab/base/libnewsrec_hip.so (tools/ab_unit_from_git.sh): parity tests of the
# working tree, then the NRMS bench line alternating new / base, then the new tree's step trace.
# Usage: bash tools/passes/ab_tree_step.sh NAME "TESTS"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-ab}; mkdir -p $O
T=${2:-tests/test_news_encoder_gpu.py}
echo tests; timeout -k 10 600 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 30 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in 1 2 3; do
  echo round $i
  timeout -k 10 200 $B > $O/bench_new_$i.json 2>> $O/bench.err || exit 3
  (cd ab/base_tree && NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/base/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_old_$i.json 2>> $O/bench.err) || exit 3
done
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
