# NRMS projection weight gradient: workspace split-K vs fp32 atomics (interleaved in one process)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abpw}; mkdir -p $O
timeout -k 10 300 python tools/ab_step.py PROJ_WGRAD_WS=0 PROJ_WGRAD_WS=1 --rounds 5 --steps 30 > $O/ab.json 2> $O/err || exit 1
echo done
