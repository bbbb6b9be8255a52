# Round 4, pass k: the key-pool forward with K staged through LDS (float4 row stores, 128 VGPRs:
# three workgroups per CU again) and its grid capped by occupancy: CNN / key-pool tests, the CNN
# legs' trace and the default bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4k}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_cnn_keypool_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
