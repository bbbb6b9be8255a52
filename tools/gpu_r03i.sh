# colsum write-through partials; A/B of the big GEMM: split-store stagger (bf16x6) and 16-deep
# bf16 k-tiles (GEMM shapes), stagger in the whole step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i
mkdir -p $O
echo tests; timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; timeout -k 10 700 python tools/gemm_ab.py --libs base,ab/stagger/libnewsrec_hip.so,ab/bk16/libnewsrec_hip.so,base,ab/stagger/libnewsrec_hip.so,ab/bk16/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_dgrad_table,nrms_proj_wgrad_atomic,bert_qkv,bert_ffn2,bert_ffn1_wgrad_cs,cnn_conv_wgrad,cnn_table_dgrad > $O/ab.json 2> $O/ab.err || exit 2
B="python bench.py --steps 60 --warmup 5 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo step; for r in 1 2; do
  timeout -k 10 200 $B > $O/step_base_$r.json 2>> $O/step.err || exit 3
  NR_LIB_PATH=ab/stagger/libnewsrec_hip.so timeout -k 10 200 $B > $O/step_stagger_$r.json 2>> $O/step.err || exit 3
done
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/kt.log 2>&1 || exit 4
echo done
