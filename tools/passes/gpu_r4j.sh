# Round 4, pass j: the key-pool forward back on its round-3 kernel (plus the K store): CNN / key-pool
# tests, the CNN legs' trace and the default bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4j}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_cnn_keypool_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_model_gpu.py tests/test_step_buffers_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo ab_step; timeout -k 10 400 python tools/ab_step.py PROJ_DGRAD_KC=0,FUSED_SAVED_BWD=0 PROJ_DGRAD_KC=1,FUSED_SAVED_BWD=0 PROJ_DGRAD_KC=0,FUSED_SAVED_BWD=1 --rounds 3 --steps 20 > $O/ab_step.json 2> $O/ab_step.err || exit 9
echo pmc_xf; bash tools/pmc_passes.sh $O/pmc_xf python tools/legs_only.py xformer --steps 1 || exit 7
echo done
