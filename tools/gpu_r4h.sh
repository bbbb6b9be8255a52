# Round 4, pass h: the step-buffer and CNN tests (LSTUR input-gradient destination, transposed conv
# weight from the pack launch) and the CNN legs' kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4h}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_step_buffers_gpu.py tests/test_cnn_keypool_gpu.py tests/test_cnn_rows_gpu.py tests/test_fullsize_cnn_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo adam_ab; timeout -k 10 300 python tools/gemm_ab.py --libs base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so,base,ab/adamnt1/libnewsrec_hip.so,ab/adamnt2/libnewsrec_hip.so --cases adam_nrms > $O/adam_ab.json 2> $O/adam_ab.err || exit 2
echo done
