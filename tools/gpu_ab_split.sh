# GEMM split-cost upper bounds (timing-only debug bits) + distinct-row tests + step kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_dedup_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t10.log 2>&1 || exit 1
timeout -k 10 400 python tools/gemm_ab.py --variants "NR_GEMM_BIG=1;NR_GEMM_BIG=1,NR_GEMM_DEBUG=64;NR_GEMM_BIG=1,NR_GEMM_DEBUG=128;NR_GEMM_BIG=1,NR_GEMM_DEBUG=192;NR_GEMM_BIG=1,NR_GEMM_DEBUG=2" --cases nrms_proj_fwd,nrms_dgrad_table,nrms_proj_wgrad > gpurun_out/ab.log 2>&1 || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt2 -o run -- $B > gpurun_out/kt2.log 2>&1 || exit 3
