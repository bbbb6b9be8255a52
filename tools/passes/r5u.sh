# Round 5, pass u: the word-table gradient with only its absent rows zeroed (the dgrad stores every
# present row); parity (dedup, news encoder, full-size steps, step buffers, graphs, data parallel);
# same-process A/B; the step trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5u}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_dedup_gpu.py tests/test_news_encoder_gpu.py tests/test_fullsize_gpu.py tests/test_step_buffers_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py tests/test_model_gpu.py tests/test_row_grad_gpu.py -v -s --timeout 500 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python tools/ab_step.py ABSENT_ROWS_ZERO=0 ABSENT_ROWS_ZERO=1 --rounds 4 > $O/ab_absent.json 2> $O/ab_absent.err || exit 3
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
