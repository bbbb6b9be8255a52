# Round 6 pass e: gloo-on-device collectives probe, the fused user-pool backward A/B, the failed tests.
O=gpurun_out/r6e
mkdir -p $O
echo probe; timeout -k 10 200 python tools/gloo_cuda_probe.py > $O/gloo_probe.json 2> $O/gloo_probe.err || exit 1
echo ab; timeout -k 10 400 python tools/ab_step.py USER_POOL_BWD_FUSED=1 USER_POOL_BWD_FUSED=0 --rounds 4 --steps 30 > $O/ab_step.json 2> $O/ab_step.err || exit 2
echo tests; timeout -k 10 600 python -u -m pytest tests/test_attn_gpu.py tests/test_mind_gpu.py tests/test_step_buffers_gpu.py tests/test_model_gpu.py tests/test_seq_pool_gpu.py tests/test_fullsize_gpu.py -k "not xformer_12" -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
echo done
