# One-off: XFormer LN backward grid cap (ab/ln512, in-tree 1024, ab/ln1536, ab/ln2048), per-lib kernel
# trace of the xformer leg + alternating leg timings.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5ab}; mkdir -p $O
X="python tools/legs_only.py xformer --steps 6"
for lib in cur ln512 ln1536 ln2048; do
  if [ $lib = cur ]; then P=""; else P=$PWD/ab/$lib/libnewsrec_hip.so; fi
  NR_LIB_PATH=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- $X > $O/leg_$lib.json 2>> $O/err.log || exit 3
done
for i in 1 2; do
  for lib in cur ln1536; do
    if [ $lib = cur ]; then P=""; else P=$PWD/ab/$lib/libnewsrec_hip.so; fi
    NR_LIB_PATH=$P timeout -k 10 200 $X > $O/t_${lib}_$i.json 2>> $O/err.log || exit 4
  done
done
echo done
