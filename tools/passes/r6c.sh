# Round 6 pass c: planes GEMM A/B + tests, side-stream / form_train bench A/B, new parity tests.
O=gpurun_out/r6c
mkdir -p $O
B="python bench.py --steps 30 --warmup 20 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo gemm_tests; timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1 || exit 1
echo gemm_ab; timeout -k 10 300 python tools/gemm_ab.py --cases nrms_proj_fwd,nrms_proj_fwd_planes,nrms_proj_fwd_rplanes,split_table_planes,split_rows_planes,nrms_dgrad_table_ws,nrms_dgrad_table_kc_ws,nrms_dgrad_table_planes > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo bench_ab
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_side_$i.json 2> $O/bench_side_$i.err || exit 3
  timeout -k 10 200 $B --no-side-streams > $O/bench_noside_$i.json 2> $O/bench_noside_$i.err || exit 3
done
echo tests; timeout -k 10 900 python -u -m pytest tests/test_mind_gpu.py tests/test_step_buffers_gpu.py tests/test_attn_gpu.py tests/test_dedup_gpu.py tests/test_row_grad_gpu.py tests/test_graph_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 4
echo done
