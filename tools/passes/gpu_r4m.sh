# Round 4, pass m: key-pool backward with kb-major dWq blocks (C column split once per kb): key-pool /
# CNN tests, same-box CNN-leg A/B against the previous cnn_keypool.hip (ab/kp_old), CNN legs trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4m}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_cnn_keypool_gpu.py tests/test_fullsize_cnn_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; for r in 1 2; do
  timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 20 > $O/legs_new_$r.json 2>> $O/ab.err || exit 2
  NR_LIB_PATH=ab/kp_old/libnewsrec_hip.so timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 20 > $O/legs_old_$r.json 2>> $O/ab.err || exit 2
done
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo done
