set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/tests_all.log 2>&1; echo tests_rc=$?
tail -4 gpurun_out/tests_all.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --eval-impr 0 > gpurun_out/b12.log 2>&1; echo rc=$?
python -c "import json; d=json.loads(open('gpurun_out/b12.log').read().strip().splitlines()[-1]); print('nrms', d['value'], d['ms_per_step'], 'xformer', d['xformer']['impressions_per_s'], d['xformer']['ms_per_step'])"
