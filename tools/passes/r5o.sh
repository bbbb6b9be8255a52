# Round 5, pass o: the weight gradient beside the dgrad, launched after it (fork event at the segment
# sums): same-process A/B and the step trace; the NRMS parity tests.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5o}; mkdir -p $O
timeout -k 10 300 python tools/ab_step.py WGRAD_BESIDE_DGRAD=0 WGRAD_BESIDE_DGRAD=1 --rounds 4 > $O/ab_beside.json 2> $O/ab_beside.err || exit 3
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -k "nrms" tests/test_graph_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_eval -o run -- python bench.py --steps 2 --warmup 2 --no-cpu-baseline --config-legs 0 --xformer-steps 0 > $O/kt_eval.log 2>&1 || exit 7
echo done
