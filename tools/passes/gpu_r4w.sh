# Round 4, pass w: batch formation with the history ids beside the negative sampling: MIND batch
# tests (bit-exact against the reference's sampling), then the NRMS step's kernel trace with this
# build and with HEAD~'s mind_batch.hip (ab/fb_old), alternating.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4w}
mkdir -p $O
echo tests; timeout -k 10 300 python -u -m pytest tests/test_mind_gpu.py tests/test_fullsize_gpu.py -m gpu -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B="python bench.py --steps 20 --warmup 3 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo trace; for r in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_new_$r -o run -- $B > $O/kt_new_$r.log 2>&1 || exit 4
  NR_LIB_PATH=ab/fb_old/libnewsrec_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_old_$r -o run -- $B > $O/kt_old_$r.log 2>&1 || exit 4
done
echo done
