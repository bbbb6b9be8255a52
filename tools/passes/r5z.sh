# Round 5, pass z: BERT input-gradient GEMMs on the transposed (k-contiguous) weights: parity (BERT /
# XFormer tests, the 12-layer step vs the float64 oracle); XFormer step A/B, alternating processes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5z}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bert_gpu.py tests/test_fullsize_gpu.py -k "xformer or bert" -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  for kc in 1 0; do
    timeout -k 10 300 python tools/legs_only.py xformer --steps 5 --set bert.DGRAD_KC=$kc > $O/xf_kc${kc}_$i.json 2>> $O/xf.err || exit 3
  done
done
echo done
