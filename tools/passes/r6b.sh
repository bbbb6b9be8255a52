mkdir -p gpurun_out/r6b
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6b/gemm_tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/gemm_ab.py --cases nrms_proj_fwd,nrms_proj_fwd_planes,nrms_proj_fwd_rplanes,split_table_planes,split_rows_planes,nrms_dgrad_table_ws,nrms_dgrad_table_kc_ws,nrms_dgrad_table_planes,nrms_proj_wgrad > gpurun_out/r6b/gemm_ab.json 2> gpurun_out/r6b/gemm_ab.err || exit 2
timeout -k 10 800 python -u -m pytest tests/test_attn_gpu.py tests/test_dedup_gpu.py tests/test_row_grad_gpu.py tests/test_fullsize_gpu.py -k "not nrms_fullsize and not cnn" -m gpu -x -v --durations=15 --timeout 400 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1 || exit 3
