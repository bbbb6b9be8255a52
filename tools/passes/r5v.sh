# Round 5, pass v: dK = W K from the key rows already in registers (no spill now) and the
# coalesced absent-row zeroing: parity; NRMS step vs ab/base (HEAD before), alternating; the trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5v}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_dedup_gpu.py tests/test_news_encoder_gpu.py tests/test_fullsize_gpu.py -k "not xformer" -v -s --timeout 500 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_new_$i.json 2>> $O/bench.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_old_$i.json 2>> $O/bench.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
