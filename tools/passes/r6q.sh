# Round 6 pass q: bf16-stored operands (NR_KCONTIG_BF16) on the big kernel: parity, GEMM timing.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6q; mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,base --cases cnn_tap_proj,cnn_tap_proj_h,cnn_table_dgrad_store,cnn_table_dgrad_store_h,cnn_table_dgrad_kc > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo done
