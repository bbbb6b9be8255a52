# Round 4, pass o: same-box XFormer step A/B of the attention backward's register bound (two waves
# per SIMD: NR_ATTN_BWDQ_WAVES / NR_ATTN_BWDKV_WAVES builds in ab/), then the BERT tests of each build.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4o}
mkdir -p $O
echo ab; for r in 1 2; do
  for v in base q2 kvq2; do
    if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=ab/$v/libnewsrec_hip.so; fi
    timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}_$r.json 2>> $O/ab.err || exit 2
  done
done
unset NR_LIB_PATH
echo tests; for v in q2 kvq2; do
  NR_LIB_PATH=ab/$v/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || exit 1
done
echo done
