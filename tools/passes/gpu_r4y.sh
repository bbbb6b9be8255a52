# Round 4, pass y: same-box XFormer step A/B of the BERT LayerNorm backward's grid cap (1024
# workgroups at HEAD; ab/g512, g2048, g4096): fewer caps = more rows per wave, more = more dgamma /
# dbeta atomics; then the XFormer kernel trace of the best-looking build is read from the step times.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4y}
mkdir -p $O
echo ab; for r in 1 2; do
  for v in base g512 g2048 g4096; do
    if [ $v = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=ab/$v/libnewsrec_hip.so; fi
    timeout -k 10 200 python tools/legs_only.py xformer --steps 5 > $O/xf_${v}_$r.json 2>> $O/ab.err || exit 2
  done
done
echo done
