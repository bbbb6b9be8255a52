# Round 4, pass e: same-box A/B of the plain weight gradient (MN x MN) k-tile: in-tree vs no A-fragment
# prefetch vs the round-3 guards vs both vs round 3 (ab/base), on the BERT weight-gradient shapes.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4e}
mkdir -p $O
L=base,ab/noapf/libnewsrec_hip.so,ab/guard/libnewsrec_hip.so,ab/both/libnewsrec_hip.so,ab/base/libnewsrec_hip.so
echo gemm_ab; timeout -k 10 500 python tools/gemm_ab.py --libs $L,$L --cases bert_ffn1_wgrad_cs,bert_ffn2_wgrad_cs,bert_qkv_wgrad_cs,nrms_proj_wgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo done
