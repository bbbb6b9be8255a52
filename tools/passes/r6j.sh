# Round 6 pass j: what dropout costs in the NRMS step (p = 0.2 vs 0, one process, interleaved), and the
# p = 0 step's kernel trace next to pass h's p = 0.2 trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6j; mkdir -p $O
echo ab; timeout -k 10 400 python tools/ab_step.py bench.DROPOUT_P=0.2 bench.DROPOUT_P=0.0 --rounds 4 --steps 30 > $O/ab_step.json 2> $O/ab_step.err || exit 1
echo trace; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/ab_step.py bench.DROPOUT_P=0.0 --rounds 1 --steps 5 > $O/kt.log 2>&1 || exit 2
echo done
