# Round 6 pass g: PMC of the configs[1] bf16 leg (its three bf16 GEMMs) and of the NRMS step
# (attention backward kernels, projection GEMMs), each counter group in its own rocprofv3 pass.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
echo pmc_bf16; bash tools/pmc_passes.sh $O/pmc_bf16 python tools/legs_only.py cnn_attn_bf16 --steps 3 || exit 1
echo pmc_nrms; bash tools/pmc_passes.sh $O/pmc_nrms python bench.py --steps 3 --warmup 2 --eval-impr 0 --config-legs 0 --xformer-steps 0 --no-cpu-baseline || exit 2
echo kt_bf16; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_bf16 -o run -- python tools/legs_only.py cnn_attn_bf16 --steps 5 > $O/kt_bf16.log 2>&1 || exit 3
echo done
