# balanced split-K wgrad: GEMM tests, full-size parity, bench line + kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d
mkdir -p $O
echo tests; timeout -k 10 600 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_fullsize_gpu.py tests/test_gemm_split_gpu.py tests/test_gemm_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; timeout -k 10 300 python tools/gemm_ab.py --libs base,ab/bn256/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_proj_wgrad > $O/ab.json 2>&1 || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 3
echo bench; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 4
echo done
