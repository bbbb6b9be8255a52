# Iteration check: a pytest selection, the default-config NRMS bench line, a kernel trace of it, and
# optional GEMM A/B over library builds (comma-separated .so paths for tools/gemm_ab.py --libs).
# Usage: bash tools/gpu_iter.sh "<pytest selection>" ["base,ab/x/libnewsrec_hip.so"]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/iter
mkdir -p $O
echo tests; timeout -k 10 500 python -u -m pytest $1 -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 2
echo bench; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 3
if [ -n "$2" ]; then echo ab; timeout -k 10 600 python tools/gemm_ab.py --libs "$2" --cases nrms_proj_fwd,nrms_dgrad_table_kc,nrms_proj_wgrad > $O/ab.json 2>&1 || exit 4; fi
echo done
