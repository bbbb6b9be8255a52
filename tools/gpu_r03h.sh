# kernel-count trims (in-kernel RNG / cursor / Adam-step advances, one-launch colsum, static loss
# gradient, atomic NRMS wgrad): the touched tests, graph/dist tests, bench line, step trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03h
mkdir -p $O
echo tests; timeout -k 10 900 python -u -m pytest tests/test_mind_gpu.py tests/test_model_gpu.py tests/test_gemm_big_gpu.py tests/test_dedup_gpu.py tests/test_graph_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_dist_gpu.py tests/test_bert_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo bench; timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo done
