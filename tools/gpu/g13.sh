set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1; echo rc=$?
tail -1 gpurun_out/bench.log
