# Round 4, pass b: the -m gpu suite, the default bench line, kernel traces (NRMS graphed steps,
# CNN legs, XFormer) and PMC passes (NRMS step, CNN legs).  Output under gpurun_out/${1:-r4b}/.
# A failing test (pytest exit 1) does not stop the pass; a crash, abort or time limit does.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4b}
mkdir -p $O
echo gemm_ab; timeout -k 10 300 python tools/gemm_ab.py --libs base,ab/ilv2/libnewsrec_hip.so,base,ab/ilv2/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_proj_wgrad,nrms_dgrad_table,nrms_dgrad_table_kc,cnn_tap_proj,bert_qkv,bert_ffn2 > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo ab_dgrad; timeout -k 10 300 python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 4 --steps 20 > $O/ab_dgrad.json 2> $O/ab_dgrad.err || exit 9
echo tests; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit 1
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 20 --warmup 3 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo legs; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 5 > $O/kt_legs.log 2>&1 || exit 5
echo xf; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 6
B3="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo pmc; bash tools/pmc_passes.sh $O/pmc $B3 || exit 7
echo pmc_legs; bash tools/pmc_passes.sh $O/pmc_legs python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 3 || exit 8
echo done
