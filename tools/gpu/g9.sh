set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_split_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t9.log 2>&1; echo tests_rc=$?
tail -3 gpurun_out/t9.log
timeout -k 10 200 python -u tools/split_probe.py > gpurun_out/split_probe.log 2>&1; echo probe_rc=$?
