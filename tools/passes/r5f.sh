# Round 5, pass f: parity tests of the new paths, the XFormer keep-bit A/B (same box, sequential
# processes, alternating), the NRMS dgrad k-contiguous A/B with its kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5f}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_bert_gpu.py tests/test_row_grad_gpu.py tests/test_attn_gpu.py tests/test_fullsize_gpu.py::test_xformer_12_layers_step_vs_oracle tests/test_fullsize_cnn_gpu.py::test_bf16_cnn_attn_fullsize_step_vs_oracle -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  for kb in 1 0; do
    timeout -k 10 200 python tools/legs_only.py xformer --steps 5 --set bert.ATTN_KEEP_BITS=$kb > $O/xf_kb${kb}_$i.json 2>> $O/xf.err || exit 2
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 3
timeout -k 10 300 python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 4 > $O/ab.json 2> $O/ab.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 1 --steps 10 > $O/kt.log 2>&1 || exit 5
echo done
