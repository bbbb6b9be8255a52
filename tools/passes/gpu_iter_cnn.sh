# CNN-family iteration: fused key-pool tests, the CNN golden / rows / full-size parity tests, the four
# CNN legs timed (graphed) and a kernel trace of them.  Output under gpurun_out/${1:-cnn}/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cnn}
mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_cnn_keypool_gpu.py tests/test_model_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py tests/test_row_grad_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo legs; timeout -k 10 300 python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 20 > $O/legs.json 2> $O/legs.err || exit 2
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 3
echo done
