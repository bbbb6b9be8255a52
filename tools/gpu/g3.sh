set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_bert.py --model xformer > gpurun_out/bx.log 2>&1
timeout -k 10 300 python -u tools/bench_bert.py --model plm --steps 3 > gpurun_out/bp.log 2>&1
tail -2 gpurun_out/bx.log gpurun_out/bp.log
