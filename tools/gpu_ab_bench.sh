# A/B of the NRMS bench line under env variants: bash tools/gpu_ab_bench.sh "VAR=a" "VAR=b" ...
# (each variant one bench process; results in gpurun_out/abb/<i>.json)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/abb
mkdir -p $O
i=0
for v in "$@"; do
  echo "variant $i: $v"
  env $v timeout -k 10 200 python bench.py --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline > $O/$i.json 2> $O/$i.err || exit 1
  i=$((i+1))
done
