# Round 5, pass t: the fixed single-row tests and the PROBE hook-owned replay test.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dedup_gpu.py tests/test_step_buffers_gpu.py -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"
echo done
