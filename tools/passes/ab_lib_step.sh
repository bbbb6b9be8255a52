# A library change against ab/base/libnewsrec_hip.so (the build before it, copied there by hand):
# big-GEMM parity, the full-size NRMS / XFormer steps vs the oracle, graph replays; same-box A/B of
# GEMM shapes (tools/gemm_ab.py) and of the NRMS step (bench.py under NR_LIB_PATH, alternating);
# the step trace.  Round 5 used it for the table dgrad's workspace tail (profiles/r05_l_*).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_fullsize_gpu.py tests/test_step_buffers_gpu.py tests/test_graph_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 400 python tools/gemm_ab.py --libs base,base --cases nrms_dgrad_table,nrms_dgrad_table_ws,nrms_proj_fwd,nrms_proj_wgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_new_$i.json 2>> $O/bench.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_old_$i.json 2>> $O/bench.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
