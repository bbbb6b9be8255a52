# Round 5, pass p: the fast eval's MHA user encoder + pooling in one launch (nr_mha_user_pool_fwd):
# kernel parity, the eval / model tests, same-process A/B of the eval leg, and its trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5p}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_gpu.py tests/test_mind_gpu.py tests/test_model_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 400 python tools/eval_ab.py USER_POOL_FUSED=0 USER_POOL_FUSED=1 --rounds 2 > $O/eval_ab.json 2> $O/eval_ab.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_eval -o run -- python bench.py --steps 2 --warmup 2 --no-cpu-baseline --config-legs 0 --xformer-steps 0 > $O/kt_eval.log 2>&1 || exit 7
echo done
