set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/tests_all.log 2>&1; echo tests_rc=$?
tail -4 gpurun_out/tests_all.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1; echo bench_rc=$?
tail -1 gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bprof -o b -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eval-impr 0 --xformer-steps 3 > gpurun_out/bprof.log 2>&1; echo prof_rc=$?
ls gpurun_out/bprof
