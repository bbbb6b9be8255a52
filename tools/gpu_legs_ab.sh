# A/B of GEMM routing env switches on config legs: bash tools/gpu_legs_ab.sh "leg ..." "ENV=V ENV2=V;ENV=V;..."
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/legs
mkdir -p $O
IFS=';' read -ra VS <<< "$2"
i=0
for v in "${VS[@]}"; do
  echo "variant $i: $v" >> $O/legs.txt
  env $v timeout -k 10 240 python tools/legs_only.py $1 --steps 20 >> $O/legs.txt 2>> $O/legs.err || exit 1
  i=$((i+1))
done
