# Round 5, pass q: nr_mha_user_pool_fwd parity (fixed test) and the eval / model tests; six waves per
# impression with O held for the L real slots (two workgroups per CU) vs twelve (ab/up12).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_gpu.py tests/test_mind_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  timeout -k 10 300 python tools/eval_ab.py USER_POOL_FUSED=1 --rounds 2 > $O/eval_new_$i.json 2>> $O/eval.err || exit 3
  NR_LIB_PATH=$PWD/ab/up12/libnewsrec_hip.so timeout -k 10 300 python tools/eval_ab.py USER_POOL_FUSED=1 --rounds 2 > $O/eval_old_$i.json 2>> $O/eval.err || exit 3
done
echo done
