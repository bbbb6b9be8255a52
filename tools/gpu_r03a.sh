# round-3 GPU pass: new tests, full -m gpu suite, default bench line, kernel trace, PMC of the
# projection GEMMs, RCCL two-ranks-on-one-GPU probe.  Output under gpurun_out/r03a/.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03a
mkdir -p $O
echo new; timeout -k 10 600 python -u -m pytest tests/test_fullsize_cnn_gpu.py tests/test_dist_gpu.py -m gpu -x -v -s --timeout 500 --timeout-method thread > $O/new.log 2>&1 || exit 1
echo all; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1 || exit 2
echo bench; timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 3
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 4
echo pmc; bash tools/pmc_passes.sh $O/pmc $B || exit 5
echo rccl; timeout -k 10 120 python tools/rccl_shared_probe.py > $O/rccl.log 2>&1; echo "rccl rc=$?" >> $O/rccl.log
echo ab; timeout -k 10 400 python tools/gemm_ab.py --libs base,ab/bn128/libnewsrec_hip.so,ab/bn256/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_dgrad_table,nrms_proj_wgrad > $O/ab.json 2>&1 || exit 6
echo done
