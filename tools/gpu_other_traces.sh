# Kernel-trace summaries of the LSTUR / GRU config legs and the XFormer train step (profiles/).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/other
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_rnn -o run -- python tools/legs_only.py cnn_lstur cnn_gru --steps 5 > $O/kt_rnn.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_xf -o run -- python tools/bench_bert.py --model xformer --steps 3 --warmup 1 > $O/kt_xf.log 2>&1 || exit 2
