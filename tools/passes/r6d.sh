# Round 6 pass d: same-process step A/Bs (k-contiguous table dgrad, fused user pool), then the new tests.
O=gpurun_out/r6d
mkdir -p $O
echo ab; timeout -k 10 400 python tools/ab_step.py PROJ_DGRAD_KC=0,encoders.USER_POOL_FUSED=1 PROJ_DGRAD_KC=1,encoders.USER_POOL_FUSED=1 PROJ_DGRAD_KC=0,encoders.USER_POOL_FUSED=0 --rounds 4 --steps 30 > $O/ab_step.json 2> $O/ab_step.err || exit 1
echo tests; timeout -k 10 800 python -u -m pytest tests/test_mind_gpu.py tests/test_attn_gpu.py tests/test_step_buffers_gpu.py tests/test_row_grad_gpu.py tests/test_dedup_gpu.py tests/test_gemm_big_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
echo dist; timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -m gpu -q -k "shard or real_model" --timeout 400 --timeout-method thread > $O/dist.log 2>&1; echo "dist rc=$?"
echo done
