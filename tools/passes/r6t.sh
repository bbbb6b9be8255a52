# dS-tile attention backward (bwd_kv stores dS, bwd_q reads it): BERT attention parity, the 12-layer
# XFormer step vs the oracle, then the XFormer leg alternating the in-tree build against ab/<v> builds
# (ab/old = the build before it).  Usage: bash tools/passes/r6t.sh OUT "v1 v2" [ROUNDS]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r6t}; mkdir -p $O
VARS=${2:-old}; R=${3:-3}
timeout -k 10 600 python -u -m pytest tests/test_bert_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_bert.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -x -q -k xformer --timeout 400 --timeout-method thread > $O/tests_xf.log 2>&1 || exit 1
for v in $VARS; do
  [ $v = old ] && continue
  NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 600 python -u -m pytest tests/test_bert_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_bert_$v.log 2>&1 || exit 1
done
for i in $(seq 1 $R); do
  echo round $i
  timeout -k 10 300 python tools/legs_only.py xformer --steps 10 > $O/xf_new_$i.json 2>> $O/xf.err || exit 3
  for v in $VARS; do
    NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 300 python tools/legs_only.py xformer --steps 10 > $O/xf_${v}_$i.json 2>> $O/xf.err || exit 3
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/legs_only.py xformer --steps 5 > $O/kt.log 2>&1 || exit 6
for v in $VARS; do
  NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v/libnewsrec_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python tools/legs_only.py xformer --steps 5 > $O/kt_$v.log 2>&1 || exit 6
done
echo done
