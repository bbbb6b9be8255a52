set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke_rc=$?; tail -1 gpurun_out/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof2 -o n -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eval-impr 0 --xformer-steps 0 --config-legs 0 > gpurun_out/nprof2.log 2>&1; echo prof_rc=$?
