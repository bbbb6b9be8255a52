# same-box A/B: user-encoder dgrad split-K (1 / 2 / 3) on the HEAD library and on a SEG_BATCH=8 build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-abseg}; mkdir -p $O
echo tests; timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py tests/test_user_split_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo ab; timeout -k 10 300 python tools/ab_step.py USER_DGRAD_SPLIT=1 USER_DGRAD_SPLIT=2 USER_DGRAD_SPLIT=3 --rounds 4 --steps 30 > $O/ab_base.json 2> $O/ab.err || exit 2
NR_LIB_PATH=ab/seg8/libnewsrec_hip.so timeout -k 10 300 python tools/ab_step.py USER_DGRAD_SPLIT=1 USER_DGRAD_SPLIT=2 --rounds 4 --steps 30 > $O/ab_seg8.json 2>> $O/ab.err || exit 3
timeout -k 10 300 python tools/ab_step.py USER_DGRAD_SPLIT=1 USER_DGRAD_SPLIT=2 --rounds 4 --steps 30 > $O/ab_base2.json 2>> $O/ab.err || exit 4
echo done
