# Round 5, pass j: the 12-layer XFormer step vs the float64 oracle at the milder init; the NRMS step's
# kernel trace with the table dgrad on the k-contiguous (transposed) weight and without, one process.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py::test_xformer_12_layers_step_vs_oracle -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_kc -o run -- python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 2 --steps 20 > $O/kt_kc.log 2>&1 || exit 6
echo done
