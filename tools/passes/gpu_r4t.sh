# Round 4, pass t: the key-pool unit tests with the multi-title-per-workgroup forward case.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4t}
mkdir -p $O
echo tests; timeout -k 10 400 python -u -m pytest tests/test_cnn_keypool_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
echo done
