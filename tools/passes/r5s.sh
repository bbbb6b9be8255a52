# Round 5, pass s: tokens alone in their distinct row's segment write their gradient row straight to the
# per-distinct-row sums (nr_mha_pool_bwd seg_off + nr_segment_rows_sum_multi): parity; same-process A/B.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5s}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_dedup_gpu.py tests/test_news_encoder_gpu.py tests/test_fullsize_gpu.py tests/test_step_buffers_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py tests/test_model_gpu.py -v -s --timeout 500 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python tools/ab_step.py SINGLE_ROWS_DIRECT=0 SINGLE_ROWS_DIRECT=1 --rounds 4 > $O/ab_direct.json 2> $O/ab_direct.err || exit 3
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
