# Round 4, pass q: same-box XFormer step A/B of the attention dK/dV kernel bounded to two waves per SIMD
# (own K / V rows held fp32 and split per tile; ab/kv2r: 256 VGPRs, 9 spilled), then the BERT tests of that build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4q}
mkdir -p $O
echo ab; for r in 1 2; do
  for v in base kv2r; do
    if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=ab/$v/libnewsrec_hip.so; fi
    timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}_$r.json 2>> $O/ab.err || exit 2
  done
done
unset NR_LIB_PATH
echo tests; NR_LIB_PATH=ab/kv2r/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_kv2r.log 2>&1 || exit 1
echo done
