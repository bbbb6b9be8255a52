set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2; do
  NR_SPLIT_KERNEL=$v timeout -k 10 120 python -u tools/split_probe.py > gpurun_out/sk_$v.log 2>&1 || echo "fail $v"
  python - $v <<'PY'
import json, sys
s = open('gpurun_out/sk_%s.log' % sys.argv[1]).read()
d = json.loads(s[s.index('{'):])
print(sys.argv[1], ' '.join('%s=%.1f' % (k[:14], v['bf16x6']['tflops']) for k, v in d.items() if k != 'accuracy'), d['accuracy']['bf16x6']['max_abs_err'])
PY
done
NR_SPLIT_KERNEL=2 timeout -k 10 300 python -u -m pytest tests/test_gemm_split_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t18.log 2>&1; echo tests_rc=$?; tail -2 gpurun_out/t18.log
