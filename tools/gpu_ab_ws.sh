# bf16 conv weight gradient: workspace split-K vs fp32 atomics (same box, alternating), + CNN tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abws}; mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_cnn_rows_gpu.py tests/test_model_gpu.py tests/test_fullsize_cnn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python tools/legs_only.py cnn_attn_bf16 --steps 40 --set WGRAD_WS_BF16=1 > $O/ws1_$r.json 2>> $O/err || exit 2
  timeout -k 10 200 python tools/legs_only.py cnn_attn_bf16 --steps 40 --set WGRAD_WS_BF16=0 > $O/ws0_$r.json 2>> $O/err || exit 3
done
echo done
