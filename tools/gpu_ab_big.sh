# A/B of big-tile GEMM builds (ab/<name>/libnewsrec_hip.so, tools/build_big_variant.sh) against the
# in-tree build on the NRMS projection shapes, after the GEMM correctness tests of the in-tree build.
# Usage: bash tools/gpu_ab_big.sh "name1 name2 ..." [extra variants ';'-separated]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/abbig
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_big_gpu.py tests/test_gemm_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
V="NR_GEMM_BIG=1"
for n in $1; do V="$V;NR_LIB_PATH=$GRAFT_REPO_ROOT/ab/$n/libnewsrec_hip.so"; done
[ -n "$2" ] && V="$V;$2"
timeout -k 10 600 python tools/gemm_ab.py --variants "$V" --cases nrms_proj_fwd,nrms_dgrad_table,nrms_dgrad_table_kc,nrms_proj_wgrad > $O/ab.json 2>&1 || exit 2
