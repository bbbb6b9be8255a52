# Round 4, pass v: same-box A/B of the segment-sum fix pass at 256 threads per workgroup (ab/sf256,
# NR_SEGFIX_THREADS=256: four times the workgroups over the distinct rows) against HEAD's 1024: the
# NRMS step (bench.py's NRMS line only) and the CNN legs, interleaved; then the dedup / CNN-row tests
# of the variant.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4v}
mkdir -p $O
B="python bench.py --steps 40 --warmup 10 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
echo ab; for r in 1 2 3; do
  for v in base sf256; do
    if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=ab/$v/libnewsrec_hip.so; fi
    timeout -k 10 200 $B > $O/nrms_${v}_$r.json 2>> $O/ab.err || exit 2
    timeout -k 10 200 python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 20 > $O/legs_${v}_$r.json 2>> $O/ab.err || exit 2
  done
done
unset NR_LIB_PATH
echo tests; NR_LIB_PATH=ab/sf256/libnewsrec_hip.so timeout -k 10 300 python -u -m pytest tests/test_dedup_gpu.py tests/test_cnn_rows_gpu.py -m gpu -q --timeout 200 --timeout-method thread > $O/tests_sf256.log 2>&1 || exit 1
echo done
