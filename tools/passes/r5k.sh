# Round 5, pass k: the head backward's dK = W K from the key rows already in registers (staged
# through the transpose tile; no second key-row load): parity (news encoder, full-size NRMS, step
# buffers) and the 12-layer XFormer step; same-box A/B of the NRMS step against ab/base (HEAD before
# the change); the k-contiguous dgrad A/B trace; the step trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5k}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py tests/test_news_encoder_gpu.py tests/test_step_buffers_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_new_$i.json 2>> $O/bench.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_old_$i.json 2>> $O/bench.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_kc -o run -- python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 2 --steps 20 > $O/kt_kc.log 2>&1 || exit 7
echo done
