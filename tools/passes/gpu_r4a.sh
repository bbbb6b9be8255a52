# Round 4, pass a: a same-box GEMM A/B (in-tree build vs ab/ilv = interleaved split-stores, ab/cf =
# conflict-free split stores only, ab/base = the round-3 GEMM units), the -m gpu suite, the default
# bench line, kernel traces of the NRMS step and the CNN legs, PMC passes of the NRMS step.
# A failing test (pytest exit 1) does not stop the pass; a crash, abort or time limit does.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4a}
mkdir -p $O
echo gemm_ab; timeout -k 10 500 python tools/gemm_ab.py --libs base,ab/ilv/libnewsrec_hip.so,ab/cf/libnewsrec_hip.so,ab/base/libnewsrec_hip.so,base,ab/ilv/libnewsrec_hip.so,ab/cf/libnewsrec_hip.so,ab/base/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_proj_dgrad,nrms_dgrad_table,nrms_proj_wgrad,cnn_tap_proj,bert_qkv,bert_ffn2,user_fwd > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo tests; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo ab_bwd; timeout -k 10 300 python tools/ab_step.py FUSED_SAVED_BWD=0 FUSED_SAVED_BWD=1 --rounds 4 --steps 20 > $O/ab_bwd.json 2> $O/ab_bwd.err || exit 7
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo pmc; bash tools/pmc_passes.sh $O/pmc $B || exit 6
echo done
