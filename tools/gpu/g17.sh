set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --eval-impr 20000 > gpurun_out/dist2.log 2>&1; echo rc=$?
tail -2 gpurun_out/dist2.log | cut -c1-600
