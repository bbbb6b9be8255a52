set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nprof -o n -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --eval-impr 0 --xformer-steps 0 > gpurun_out/nprof.log 2>&1; echo prof_rc=$?
bash tools/pmc_passes.sh gpurun_out/pmc python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --eval-impr 0 --xformer-steps 0; echo pmc_rc=$?
ls gpurun_out/pmc
