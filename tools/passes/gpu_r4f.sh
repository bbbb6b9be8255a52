# Round 4, pass f: same-box A/B of the MN-contiguous loaders without the always-false thread guards
# (a branch-free k-tile for the weight gradients): in-tree vs the interleave on MN x MN (ab/ilv33)
# vs round 3 (ab/base); then the XFormer trace and the GEMM unit tests.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4f}
mkdir -p $O
L=base,ab/ilv33/libnewsrec_hip.so,ab/base/libnewsrec_hip.so
echo gemm_ab; timeout -k 10 500 python tools/gemm_ab.py --libs $L,$L --cases bert_ffn1_wgrad_cs,bert_ffn2_wgrad_cs,bert_qkv_wgrad_cs,nrms_proj_wgrad,cnn_conv_wgrad,user_wgrad > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
echo gemm_tests; timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_big_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/gemm_tests.log 2>&1 || exit 1
echo xf; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/legs_only.py xformer --steps 3 > $O/kt_xf.log 2>&1 || exit 6
echo done
