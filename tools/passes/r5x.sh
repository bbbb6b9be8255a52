# Round 5, pass x: fast-eval predict batch 2048 vs 8192 impressions (host loop amortisation).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5x}; mkdir -p $O
timeout -k 10 500 python tools/eval_ab.py bench.EVAL_BATCH_IMPR=2048 bench.EVAL_BATCH_IMPR=8192 bench.EVAL_BATCH_IMPR=16384 --rounds 2 > $O/eval_batch_ab.json 2> $O/eval.err || exit 3
echo done
