# NRMS iteration: graph / dedup / full-size tests, the default-config bench line, a kernel trace of the step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-nrms}
mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_dedup_gpu.py tests/test_fullsize_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo bench; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 3
echo done
