# Round 4, pass h: the step-buffer / CNN / key-pool tests (LSTUR input-gradient destination, transposed
# conv weight from the pack launch, the planes key-pool forward and the saved K), the CNN legs' trace,
# A/B: Adam with nontemporal accesses, the interleave on the dgrad operand pair (ab/ilv03); then the
# -m gpu suite, the default bench line and the NRMS graphed-step trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4h}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_step_buffers_gpu.py tests/test_cnn_keypool_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo adam_ab; timeout -k 10 300 python tools/gemm_ab.py --libs base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so,base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so --cases adam_nrms > $O/adam_ab.json 2> $O/adam_ab.err || exit 2
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/ilv03/libnewsrec_hip.so,base,ab/ilv03/libnewsrec_hip.so --cases nrms_proj_dgrad,nrms_dgrad_table,bert_ffn2_dgrad,bert_qkv_dgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
for v in attnpf xfall; do
  echo tests_$v; NR_LIB_PATH=$PWD/ab/$v/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/${v}_tests.log 2>&1 || exit 1
done
for i in 1; do for v in base attnpf lnpf xfall; do
  if [ $v = base ]; then LP=""; else LP=$PWD/ab/$v/libnewsrec_hip.so; fi
  echo xf_$v; NR_LIB_PATH=$LP timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}_$i.json 2> $O/xf_${v}_$i.err || exit 8
done; done
echo all_tests; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread > $O/all_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 20 --warmup 3 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo done
