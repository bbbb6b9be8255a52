# Round 5, pass i: the odd/even two-tile k-loop for bf16 (one-product) big-GEMM units -- parity of
# the big GEMM tests and the 12-layer XFormer step; same-box A/B against ab/base (HEAD before the
# change) on the bf16 / bf16x6 GEMM shapes and the CNN legs (configs[1] bf16 uses these units).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5i}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_fullsize_gpu.py::test_xformer_12_layers_step_vs_oracle tests/test_step_buffers_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 600 python tools/gemm_ab.py --libs base,ab/base/libnewsrec_hip.so,base,ab/base/libnewsrec_hip.so --cases cnn_tap_proj,cnn_conv_wgrad,cnn_table_dgrad,nrms_proj_fwd,nrms_proj_wgrad,bert_qkv,bert_ffn1_wgrad_cs,bert_qkv_dgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
for i in 1 2; do
  timeout -k 10 200 python tools/legs_only.py cnn_attn_bf16 cnn_attn --steps 20 > $O/legs_new_$i.json 2>> $O/legs.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 python tools/legs_only.py cnn_attn_bf16 cnn_attn --steps 20 > $O/legs_old_$i.json 2>> $O/legs.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn_bf16 --steps 10 > $O/kt_legs.log 2>&1 || exit 6
echo done
