# A pytest selection, then a kernel trace of the given config legs: bash tools/gpu_leg_trace.sh "<tests>" "leg ..."
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/legtrace
mkdir -p $O
timeout -k 10 500 python -u -m pytest $1 -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/legs_only.py $2 --steps 5 > $O/kt.log 2>&1 || exit 2
