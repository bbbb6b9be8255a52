# Round 4, pass p: same-box XFormer step A/B of the attention forward bounded to three waves per SIMD
# (NR_ATTN_FWD_WAVES=3 build in ab/f3: 168 VGPRs, 13 / 5 spilled), then the BERT tests of that build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4p}
mkdir -p $O
echo ab; for r in 1 2; do
  for v in base f3; do
    if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=ab/$v/libnewsrec_hip.so; fi
    timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}_$r.json 2>> $O/ab.err || exit 2
  done
done
unset NR_LIB_PATH
echo tests; NR_LIB_PATH=ab/f3/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_f3.log 2>&1 || exit 1
echo done
