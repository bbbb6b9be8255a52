# key-pool iteration: its tests, the probe, the CNN legs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-kp}
mkdir -p $O
echo tests; timeout -k 10 300 python -u -m pytest tests/test_cnn_keypool_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo probe; timeout -k 10 120 python tools/keypool_probe.py > $O/probe.json 2> $O/probe.err || exit 2
echo legs; timeout -k 10 300 python tools/legs_only.py cnn_attn cnn_attn_bf16 cnn_lstur cnn_gru --steps 20 > $O/legs.json 2> $O/legs.err || exit 3
echo done
echo kt; timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python tools/keypool_probe.py > $O/kt.log 2>&1 || exit 4
echo done2
