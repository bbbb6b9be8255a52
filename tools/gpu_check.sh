# quick GPU check: the given pytest selection, then the NRMS bench line and a kernel trace of it
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SEL=${1:-tests}
timeout -k 10 400 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tc.log 2>&1 || exit 1
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktc -o run -- $B > gpurun_out/ktc.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > gpurun_out/bc.json 2> gpurun_out/bc.err || exit 3
