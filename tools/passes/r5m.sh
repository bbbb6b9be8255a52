# Round 5, pass m: 12-layer XFormer step vs the float64 oracle (starting-point fix); graph launch gap
# (events around replays, and two steps per graph); k-contiguous dgrad A/B with the workspace tail;
# PMC passes of the NRMS bench for the projection GEMMs (the bench line's traffic figures).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py::test_xformer_12_layers_step_vs_oracle -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python tools/graph_gap.py > $O/graph_gap.json 2> $O/graph_gap.err || exit 2
timeout -k 10 300 python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 4 > $O/ab_kc.json 2> $O/ab_kc.err || exit 3
bash tools/pmc_passes.sh $O/pmc python bench.py --steps 5 --warmup 3 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0 || exit 4
for k in "proj_fwd:gemm_big_kernel<1, 0, true, 3" "proj_dgrad:gemm_big_kernel<0, 3, true, 3" "proj_wgrad:gemm_big_kernel<3, 4, false, 3" "tail_reduce:tail_reduce_kernel" "splitk_reduce:splitk_reduce_kernel"; do
  python tools/summarize_pmc.py $O/pmc "${k#*:}" $O/pmc_${k%%:*}.json > /dev/null || exit 5
done
echo done
