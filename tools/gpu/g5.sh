set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/split_probe.py > gpurun_out/split_probe.log 2>&1; echo probe_rc=$?
NR_GEMM_PREC=bf16x6 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_bf16x6.log 2>&1; echo tests_rc=$?
tail -5 gpurun_out/tests_bf16x6.log
NR_GEMM_PREC=bf16x6 timeout -k 10 300 python -u bench.py --no-cpu-baseline --eval-impr 0 > gpurun_out/bench_bf16x6.log 2>&1; echo bench_rc=$?
NR_GEMM_PREC=bf16x6 timeout -k 10 300 python -u tools/bench_bert.py --model xformer > gpurun_out/bx6.log 2>&1; echo bx_rc=$?
