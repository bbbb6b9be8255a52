set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/bench_final.log 2>&1; echo rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof3 -o n -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eval-impr 0 --xformer-steps 0 --config-legs 0 > gpurun_out/nprof3.log 2>&1; echo prof_rc=$?
