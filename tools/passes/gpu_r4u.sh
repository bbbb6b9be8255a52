# Round 4, pass u: PMC passes over the CNN + attention legs (fp32-class and bf16) for the key-pool
# kernels of HEAD.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4u}
mkdir -p $O
echo pmc; bash tools/pmc_passes.sh $O/pmc_kp python tools/legs_only.py cnn_attn cnn_attn_bf16 --steps 2 || exit 7
echo done
