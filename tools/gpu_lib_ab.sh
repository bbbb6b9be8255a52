# A/B of library builds (ab/<name>/libnewsrec_hip.so via NR_LIB_PATH; "base" = the in-tree build):
# a pytest selection, a kernel trace and the NRMS bench line for each.
# Usage: bash tools/gpu_lib_ab.sh "<tests>" "base name1 name2 ..."
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/libab
mkdir -p $O
B="python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline"
for n in $2; do
  if [ "$n" = base ]; then unset NR_LIB_PATH; else export NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$n/libnewsrec_hip.so; fi
  echo "$n tests"; timeout -k 10 400 python -u -m pytest $1 -m gpu -x -q --timeout 300 --timeout-method thread > $O/$n.tests.log 2>&1 || exit 1
  echo "$n trace"; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- $B > $O/$n.kt.log 2>&1 || exit 2
  echo "$n bench"; timeout -k 10 300 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/$n.bench.json 2> $O/$n.bench.err || exit 3
done
echo done
