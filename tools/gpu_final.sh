# Round-end evidence: GPU tests, the default bench line, kernel-trace summaries (NRMS step, CNN legs)
# and the projection GEMM / attention PMC passes.  Output under gpurun_out/final/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/final
mkdir -p $O
echo "tests"; timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo "bench"; timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo "trace nrms"; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_nrms -o run -- $B > $O/kt_nrms.log 2>&1 || exit 3
echo "trace legs"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_legs -o run -- python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 5 > $O/kt_legs.log 2>&1 || exit 4
echo "pmc"; bash tools/pmc_passes.sh $O/pmc $B || exit 5
echo "done"
