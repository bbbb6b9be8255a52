set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_split_gpu.py tests/test_model_gpu.py tests/test_gemm_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t16.log 2>&1; echo tests_rc=$?
tail -3 gpurun_out/t16.log
timeout -k 10 300 python -u tools/legs_only.py > gpurun_out/legs.log 2>&1; echo rc=$?; tail -1 gpurun_out/legs.log
