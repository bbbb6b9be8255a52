set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lprof -o l -- python3 tools/legs_only.py > gpurun_out/lprof.log 2>&1; echo rc=$?
