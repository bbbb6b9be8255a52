set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NR_GEMM_PREC=bf16x6 timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/tests_bf16x6.log 2>&1; echo tests_rc=$?
tail -8 gpurun_out/tests_bf16x6.log
