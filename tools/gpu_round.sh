# GPU check used while iterating: full -m gpu suite, GEMM A/B on the step's projection shapes, the
# default-config NRMS bench line and a kernel trace of it (per-step table: tools/step_kernels.py).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/round
mkdir -p $O
echo "tests"; timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo "gemm"; timeout -k 10 200 python tools/gemm_ab.py --variants "NR_GEMM_BIG=1" --cases nrms_proj_fwd,nrms_dgrad_table_kc,nrms_proj_wgrad > $O/ab.json 2>&1 || exit 2
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo "trace"; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 3
echo "bench"; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 4
echo done
