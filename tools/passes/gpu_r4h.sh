# Round 4, pass h: targeted tests of this round's later changes (step buffers, CNN pack / key-pool planes
# forward / saved K) and the A/B builds: Adam nontemporal (ab/adamnt*), interleave on the dgrad pair
# (ab/ilv03), K = 480 on the big kernel (ab/kmin480), BERT attention prefetch / LN prefetch (ab/attnpf,
# ab/lnpf, ab/xfall = both + fused staging), each variant's parity tests first.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4h}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_step_buffers_gpu.py tests/test_cnn_keypool_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo adam_ab; timeout -k 10 300 python tools/gemm_ab.py --libs base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so,base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so --cases adam_nrms > $O/adam_ab.json 2> $O/adam_ab.err || exit 2
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/ilv03/libnewsrec_hip.so,ab/kmin480/libnewsrec_hip.so,base,ab/ilv03/libnewsrec_hip.so,ab/kmin480/libnewsrec_hip.so --cases nrms_proj_dgrad,nrms_dgrad_table,bert_ffn2_dgrad,bert_qkv_dgrad,cnn_table_dgrad_kc > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
for v in attnpf xfall; do
  echo tests_$v; NR_LIB_PATH=$PWD/ab/$v/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/${v}_tests.log 2>&1 || exit 1
done
for v in base attnpf lnpf xfall; do
  if [ $v = base ]; then LP=""; else LP=$PWD/ab/$v/libnewsrec_hip.so; fi
  echo xf_$v; NR_LIB_PATH=$LP timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}.json 2> $O/xf_${v}.err || exit 8
done
for v in base kmin480 base kmin480; do
  if [ $v = base ]; then LP=""; else LP=$PWD/ab/$v/libnewsrec_hip.so; fi
  echo legs_$v; NR_LIB_PATH=$LP timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 20 >> $O/legs_${v}.json 2>> $O/legs_${v}.err || exit 8
done
echo legs_trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo done
