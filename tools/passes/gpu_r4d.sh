# Round 4, pass d: the bf16-MFMA attention (bert tests first), GEMM A/B of the branch-free column sum
# on the plain weight gradient (in-tree vs ab/ilv33 vs ab/base = round 3), an XFormer kernel trace,
# the -m gpu suite, the default bench line.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4d}
mkdir -p $O
echo bert; timeout -k 10 300 python -u -m pytest tests/test_bert_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/bert_tests.log 2>&1 || exit 1
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/ilv33/libnewsrec_hip.so,ab/base/libnewsrec_hip.so,base,ab/base/libnewsrec_hip.so --cases bert_ffn1_wgrad_cs,bert_ffn1_wgrad,nrms_proj_wgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo xf; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 6
echo tests; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
echo bench; timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
