# bf16x6 conv weight gradient: workspace split-K vs fp32 atomics (same box, alternating)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abws6}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_gru --steps 40 --set WGRAD_WS_BF16X6=1 > $O/ws1_$r.json 2>> $O/err || exit 2
  timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_gru --steps 40 --set WGRAD_WS_BF16X6=0 > $O/ws0_$r.json 2>> $O/err || exit 3
done
echo done
