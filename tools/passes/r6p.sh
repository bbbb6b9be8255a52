# Round 6 pass p: the sharded-table GPU tests with the calibrated bar.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p; mkdir -p $O
echo tests; timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -k shard -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1; echo "rc=$?"
echo done
