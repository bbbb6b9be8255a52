# Same-box A/B of module switches (newsrec_amd.functions): the NRMS step interleaved in one process
# (tools/ab_step.py) and the graphed CNN legs alternating (tools/legs_only.py --set).
# Usage: bash tools/gpu_ab.sh OUT "SWITCH=0 SWITCH=1" ["leg ..."]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python tools/ab_step.py $2 --rounds 5 --steps 30 > $O/ab_nrms.json 2> $O/err || exit 1
if [ -n "$3" ]; then
  for r in 1 2; do
    for v in $2; do
      timeout -k 10 200 python tools/legs_only.py $3 --steps 40 --set $v > $O/legs_${v}_$r.json 2>> $O/err || exit 2
    done
  done
fi
echo done
