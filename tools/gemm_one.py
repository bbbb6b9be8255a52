"""Run one GEMM case of tools/gemm_ab.py `reps` times (a short program for rocprofv3 --pmc passes).
python tools/gemm_one.py nrms_proj_fwd [bf16x6|bf16] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gemm_ab  # noqa: E402

name = sys.argv[1]
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16x6"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
src = gemm_ab.CHILD.split("out = {}")[0]
src += '''
p = L.GEMM_BF16X6 if "%s" == "bf16x6" else L.GEMM_BF16
fl, fn = cases["%s"]
for _ in range(%d):
    fn(p)
torch.cuda.synchronize()
''' % (prec, name, reps)
exec(compile(src, "gemm_one", "exec"))
