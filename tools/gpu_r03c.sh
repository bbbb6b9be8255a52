# GEMM A/B: B pre-split (gemm_bg) vs both operands in LDS, on the step's shapes; NRMS step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
echo ab; timeout -k 10 400 python tools/gemm_ab.py --cases nrms_proj_fwd,nrms_proj_fwd_bs,nrms_dgrad_table,nrms_dgrad_table_bs,cnn_tap_proj,cnn_tap_proj_bs,bert_qkv,bert_qkv_bs,bert_ffn1_gelu,bert_ffn1_gelu_bs,bert_ffn2,bert_ffn2_bs > $O/ab.json 2>&1 || exit 1
echo step; timeout -k 10 300 python tools/ab_step.py SPLIT_B=1 SPLIT_B=0 --rounds 4 > $O/ab_step.json 2> $O/ab_step.err || exit 2
echo done
