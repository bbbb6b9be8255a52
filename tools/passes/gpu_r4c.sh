# Round 4, pass c: GEMM A/B of the interleave on the plain weight gradient (in-tree: off; ab/ilv33:
# on; ab/base: round 3), the -m gpu suite, the default bench line, an XFormer kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4c}
mkdir -p $O
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/ilv33/libnewsrec_hip.so,ab/base/libnewsrec_hip.so,base,ab/ilv33/libnewsrec_hip.so,ab/base/libnewsrec_hip.so --cases bert_ffn1_wgrad_cs,nrms_proj_wgrad,bert_qkv,nrms_proj_fwd > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo tests; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
echo bench; timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo xf; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 6
echo done
