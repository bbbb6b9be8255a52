# Round 5, pass g: parity tests of the round's new paths; same-box A/Bs: the branch-free bf16x6 k-loop
# (in-tree library vs ab/base = the previous commit) on the GEMM shapes and the NRMS step, the XFormer
# keep bits, the k-contiguous NRMS dgrad; the NRMS step's kernel trace.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5g}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_bert_gpu.py tests/test_row_grad_gpu.py tests/test_attn_gpu.py tests/test_fullsize_gpu.py::test_xformer_12_layers_step_vs_oracle tests/test_fullsize_cnn_gpu.py::test_bf16_cnn_attn_fullsize_step_vs_oracle tests/test_gemm_big_gpu.py -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 600 python tools/gemm_ab.py --libs base,ab/base/libnewsrec_hip.so,base,ab/base/libnewsrec_hip.so --cases nrms_proj_fwd,nrms_dgrad_table,nrms_dgrad_table_kc,nrms_proj_wgrad,bert_qkv,bert_ffn2,bert_ffn1_wgrad_cs,bert_qkv_dgrad,cnn_tap_proj > $O/gemm_ab.json 2> $O/gemm_ab.err || exit 2
B="python bench.py --steps 20 --warmup 20 --no-cpu-baseline --eval-impr 0 --config-legs 0 --xformer-steps 0"
for i in 1 2; do
  timeout -k 10 200 $B > $O/bench_new_$i.json 2>> $O/bench.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 $B > $O/bench_old_$i.json 2>> $O/bench.err || exit 3
done
for kb in 1 0; do
  timeout -k 10 200 python tools/legs_only.py xformer --steps 5 --set bert.ATTN_KEEP_BITS=$kb > $O/xf_kb${kb}.json 2>> $O/xf.err || exit 4
done
NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 200 python tools/legs_only.py xformer --steps 5 --set bert.ATTN_KEEP_BITS=0 > $O/xf_old.json 2>> $O/xf.err || exit 4
timeout -k 10 300 python tools/ab_step.py PROJ_DGRAD_KC=0 PROJ_DGRAD_KC=1 --rounds 4 > $O/ab_kc.json 2> $O/ab_kc.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 6
echo done
