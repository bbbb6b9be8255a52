# Round 5, pass y: the CNN table dgrad (K = 480) on the big kernel with the workspace tail + absent-row
# zeroing: parity (CNN full-size legs vs the oracle, goldens, dedup, graphs); CNN legs vs ab/base.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5y}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fullsize_cnn_gpu.py tests/test_cnn_rows_gpu.py tests/test_model_gpu.py tests/test_gemm_big_gpu.py tests/test_graph_gpu.py tests/test_dedup_gpu.py -v -s --timeout 600 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
for i in 1 2; do
  timeout -k 10 300 python tools/legs_only.py cnn_attn cnn_gru cnn_lstur --steps 20 > $O/legs_new_$i.json 2>> $O/legs.err || exit 3
  NR_LIB_PATH=$PWD/ab/base/libnewsrec_hip.so timeout -k 10 300 python tools/legs_only.py cnn_attn cnn_gru cnn_lstur --steps 20 > $O/legs_old_$i.json 2>> $O/legs.err || exit 3
done
echo done
