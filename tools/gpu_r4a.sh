# Round 4, pass a: the -m gpu suite, a same-box GEMM A/B (in-tree build vs the round-3 GEMM units,
# ab/base), the default bench line, a kernel trace of the NRMS step and PMC passes of it.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4a}
mkdir -p $O
echo tests; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo gemm_ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/base/libnewsrec_hip.so,base,ab/base/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_proj_dgrad,nrms_dgrad_table,nrms_proj_wgrad,cnn_tap_proj,bert_qkv,bert_ffn2,user_fwd > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo pmc; bash tools/pmc_passes.sh $O/pmc $B || exit 5
echo done
