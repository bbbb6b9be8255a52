set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bert_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/bert_tests.log 2>&1; echo rc=$?
tail -40 gpurun_out/bert_tests.log
