# B-from-global GEMM check: its kernel tests, the full-size NRMS parity, graph tests, step A/B, bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03b
mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_gemm_bg_gpu.py tests/test_fullsize_gpu.py tests/test_graph_gpu.py tests/test_dedup_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; timeout -k 10 300 python tools/ab_step.py SPLIT_B=1 SPLIT_B=0 --rounds 3 > $O/ab_step.json 2> $O/ab_step.err || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 3
echo bench; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 4
echo done
