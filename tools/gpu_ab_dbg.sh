cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab1
timeout -k 10 400 python tools/gemm_ab.py --variants "NR_GEMM_DEBUG=0;NR_GEMM_DEBUG=1;NR_GEMM_DEBUG=2;NR_GEMM_DEBUG=4;NR_GEMM_DEBUG=7;NR_GEMM_DEBUG=32" --cases nrms_proj_fwd,nrms_dgrad_table,nrms_dgrad_table_kc,nrms_proj_wgrad > gpurun_out/ab1/ab.json 2>&1
