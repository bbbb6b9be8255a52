set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base prio early both base; do
  if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=$PWD/ab_old/$v/libnewsrec_hip.so; fi
  timeout -k 10 120 python -u tools/split_probe.py > gpurun_out/sp_$v.log 2>&1 || echo "fail $v"
  python - $v <<'PY'
import json, sys
s = open('gpurun_out/sp_%s.log' % sys.argv[1]).read()
d = json.loads(s[s.index('{'):])
print(sys.argv[1], ' '.join('%s=%.1f' % (k[:14], v['bf16x6']['tflops']) for k, v in d.items() if k != 'accuracy'))
PY
done
