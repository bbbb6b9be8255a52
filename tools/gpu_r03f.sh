# dedup (fused count+scan, self-cleaning workspace) + fused head tests, priority A/B of the big
# GEMM, the bench line and a step trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f
mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_dedup_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_cnn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; timeout -k 10 500 python tools/gemm_ab.py --libs base,ab/prio_static/libnewsrec_hip.so,ab/asmsub/libnewsrec_hip.so,ab/noslp/libnewsrec_hip.so,base --cases nrms_proj_fwd,nrms_dgrad_table,nrms_proj_wgrad,bert_qkv,bert_ffn2,bert_ffn1_wgrad > $O/ab.json 2> $O/ab.err || exit 2
echo bench; timeout -k 10 400 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo done
