# Round 5, pass n: the projection weight gradient on a side stream beside the table dgrad (one
# process): parity (full-size NRMS / XFormer vs the oracle incl. the Adam check, graph replays, step
# buffers, data-parallel tests that keep the hooks' path); same-process A/B; the step trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5n}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_fullsize_gpu.py tests/test_step_buffers_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py -v -s --timeout 500 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python tools/ab_step.py WGRAD_BESIDE_DGRAD=0 WGRAD_BESIDE_DGRAD=1 --rounds 4 > $O/ab_beside.json 2> $O/ab_beside.err || exit 3
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
