set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --graph off --no-cpu-baseline --eval-impr 0 --xformer-steps 0 > gpurun_out/b_eager.log 2>&1; echo rc=$?
python -c "import json; d=json.loads(open('gpurun_out/b_eager.log').read().strip().splitlines()[-1]); print('eager', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --eval-impr 0 --xformer-steps 0 > gpurun_out/b_graph.log 2>&1; echo rc=$?
python -c "import json; d=json.loads(open('gpurun_out/b_graph.log').read().strip().splitlines()[-1]); print('graph', d['value'], d['ms_per_step'])"
