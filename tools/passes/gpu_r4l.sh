# Round 4, pass l: attention staging with the conflict-free slot mapping (bert.hip tile_slot): BERT
# tests, same-box XFormer step A/B against the previous bert.hip (ab/bert_old, built by
# tools/ab_unit_from_git.sh), XFormer kernel trace and the attention PMC passes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4l}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_bert_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; for r in 1 2; do
  timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_new_$r.json 2>> $O/ab.err || exit 2
  NR_LIB_PATH=ab/bert_old/libnewsrec_hip.so timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_old_$r.json 2>> $O/ab.err || exit 2
done
echo xf; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 6
echo pmc_xf; bash tools/pmc_passes.sh $O/pmc_xf python tools/legs_only.py xformer --steps 1 || exit 7
echo done
