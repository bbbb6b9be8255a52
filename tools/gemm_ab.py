"""A/B timing of the GEMM kernels on the step's shapes, bf16x6 and bf16: one process per library
build (NR_LIB_PATH; variant builds come from tools/build_variant*.sh, the product library has no
run-time switches).  python tools/gemm_ab.py [--libs base,ab/x/libnewsrec_hip.so] [--cases ...]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, sys, torch
sys.path.insert(0, "%s/news-recommendation-mind_amd")
from newsrec_amd import _lib as L, kernels as K, functions as F
def bench(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
dev = "cuda"; torch.manual_seed(0)
V, E, U = 30522, 768, 24576
table = torch.randn(V, E, device=dev); ids = torch.randint(1, V, (U,), device=dev)
W = torch.randn(1152, E, device=dev) / 30
Y = torch.empty(U, 1152, device=dev); dY = torch.randn(U, 1152, device=dev)
dX = torch.empty(U, E, device=dev); dW = torch.zeros(1152, E, device=dev)
T = 20832
x = torch.randn(T, 768, device=dev); wqkv = torch.randn(2304, 768, device=dev) / 30
qkv = torch.empty(T, 2304, device=dev); wi = torch.randn(3072, 768, device=dev) / 30
G = torch.empty(T, 3072, device=dev); Ub = torch.empty(T, 3072, device=dev)
wo2 = torch.randn(768, 3072, device=dev) / 50; o = torch.empty(T, 768, device=dev)
dWi = torch.zeros(3072, 768, device=dev); dbi = torch.zeros(3072, device=dev)
dWo2 = torch.zeros(768, 3072, device=dev); dbo2 = torch.zeros(768, device=dev)
dWqkv = torch.zeros(2304, 768, device=dev); dbqkv = torch.zeros(2304, device=dev)
P = torch.empty(U, 480, device=dev); w3 = torch.randn(480, E, device=dev); Pg = torch.randn(U, 480, device=dev); dw3 = torch.zeros(480, E, device=dev)
uids = torch.randperm(V - 1, device=dev)[:24600] + 1; dT = torch.zeros(V, E, device=dev); w3T = w3.t().contiguous()
dYc = torch.randn(52800, 1152, device=dev); WT = W.t().contiguous()
ux = torch.randn(1600, 384, device=dev); uw = torch.randn(768, 384, device=dev) / 20; ub = torch.randn(768, device=dev)
uy = torch.empty(1600, 768, device=dev); udy = torch.randn(1600, 768, device=dev); udx = torch.empty(1600, 384, device=dev)
udw = torch.zeros(768, 384, device=dev); udb = torch.zeros(768, device=dev); uwT = uw.t().contiguous(); m_dev = torch.tensor([24600], dtype=torch.int32, device=dev)
adam_p = [torch.randn(30522, 768, device=dev), torch.randn(1152, 768, device=dev), torch.randn(768, 384, device=dev)]
adam_s = [(q, torch.randn_like(q), torch.zeros_like(q), torch.zeros_like(q)) for q in adam_p]
def adam_step(p):
    K.adam_multi([(q, g, m, v, 1e-4, 1) for q, g, m, v in adam_s], 0.9, 0.999, 1e-8, 0.0)
cases = {
 "adam_nrms": (0, adam_step),
 "nrms_proj_fwd": (2*U*E*1152, lambda p: K.gemm_dyn(U, 1152, E, K.operand(table, L.KCONTIG, rows=ids, mapping=L.ROWS_GATHER), K.operand(W, L.KCONTIG), Y, prec=p)),
 "nrms_proj_dgrad": (2*U*E*1152, lambda p: K.gemm_dyn(U, E, 1152, K.operand(dY, L.KCONTIG), K.operand(W, L.MNCONTIG), dX, prec=p)),
 "nrms_dgrad_table": (2*24600*E*1152, lambda p: K.gemm_dyn(52800, E, 1152, K.operand(dYc, L.KCONTIG), K.operand(W, L.MNCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p)),
 "nrms_dgrad_table_kc": (2*24600*E*1152, lambda p: K.gemm_dyn(52800, E, 1152, K.operand(dYc, L.KCONTIG), K.operand(WT, L.KCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p)),
 "nrms_dgrad_table_ws": (2*24600*E*1152, lambda p: K.gemm_dyn(52800, E, 1152, K.operand(dYc, L.KCONTIG), K.operand(W, L.MNCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p, workspace=True)),
 "nrms_dgrad_table_store": (2*24600*E*1152, lambda p: K.gemm_dyn(52800, E, 1152, K.operand(dYc, L.KCONTIG), K.operand(W, L.MNCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_STORE, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p)),
 "user_fwd": (2*1600*768*384, lambda p: K.gemm(1600, 768, 384, K.operand(ux, L.KCONTIG), K.operand(uw, L.KCONTIG), uy, bias=ub, prec=p)),
 "user_dgrad": (2*1600*768*384, lambda p: K.gemm(1600, 384, 768, K.operand(udy, L.KCONTIG), K.operand(uw, L.MNCONTIG), udx, prec=p)),
 "user_dgrad_kc": (2*1600*768*384, lambda p: K.gemm(1600, 384, 768, K.operand(udy, L.KCONTIG), K.operand(uwT, L.KCONTIG), udx, prec=p)),
 "user_wgrad": (2*1600*768*384, lambda p: K.gemm(768, 384, 1600, K.operand(udy, L.MNCONTIG), K.operand(ux, L.MNCONTIG), udw, epilogue=L.EPI_ATOMIC, split_k=F._split_k(768, 384, 1600), prec=p)),
 "user_wgrad_s25": (2*1600*768*384, lambda p: K.gemm(768, 384, 1600, K.operand(udy, L.MNCONTIG), K.operand(ux, L.MNCONTIG), udw, epilogue=L.EPI_ATOMIC, split_k=25, prec=p)),
 "user_wgrad_s25_cs": (2*1600*768*384, lambda p: K.gemm(768, 384, 1600, K.operand(udy, L.MNCONTIG), K.operand(ux, L.MNCONTIG), udw, epilogue=L.EPI_ATOMIC, split_k=25, prec=p, colsum=udb)),
 "user_wgrad_cs": (2*1600*768*384, lambda p: K.gemm(768, 384, 1600, K.operand(udy, L.MNCONTIG), K.operand(ux, L.MNCONTIG), udw, epilogue=L.EPI_ATOMIC, split_k=F._split_k(768, 384, 1600), prec=p, colsum=udb)),
 "user_wgrad_s50": (2*1600*768*384, lambda p: K.gemm(768, 384, 1600, K.operand(udy, L.MNCONTIG), K.operand(ux, L.MNCONTIG), udw, epilogue=L.EPI_ATOMIC, split_k=50, prec=p)),
 "nrms_proj_wgrad": (2*U*E*1152, lambda p: K.gemm_dyn(1152, E, U, K.operand(dY, L.MNCONTIG), K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_GATHER), dW, epilogue=L.EPI_ATOMIC, split_k=F._split_k(1152, E, U), prec=p)),
 "cnn_tap_proj": (2*U*E*480, lambda p: K.gemm_dyn(U, 480, E, K.operand(table, L.KCONTIG, rows=ids, mapping=L.ROWS_GATHER), K.operand(w3, L.KCONTIG), P, prec=p)),
 "bert_qkv": (2*T*768*2304, lambda p: K.gemm(T, 2304, 768, K.operand(x, L.KCONTIG), K.operand(wqkv, L.KCONTIG), qkv, prec=p)),
 "bert_ffn1_gelu": (2*T*768*3072, lambda p: K.gemm(T, 3072, 768, K.operand(x, L.KCONTIG), K.operand(wi, L.KCONTIG), G, epilogue=L.EPI_STORE_GELU, c_rows=K.operand(Ub, L.KCONTIG), prec=p)),
 "bert_ffn2": (2*T*768*3072, lambda p: K.gemm(T, 768, 3072, K.operand(G, L.KCONTIG), K.operand(wo2, L.KCONTIG), o, prec=p)),
 "bert_ffn1_wgrad": (2*T*768*3072, lambda p: K.gemm(3072, 768, T, K.operand(G, L.MNCONTIG), K.operand(x, L.MNCONTIG), dWi, epilogue=L.EPI_ATOMIC, split_k=F._split_k(3072, 768, T), prec=p)),
 "bert_ffn1_wgrad_cs": (2*T*768*3072, lambda p: K.gemm(3072, 768, T, K.operand(G, L.MNCONTIG), K.operand(x, L.MNCONTIG), dWi, epilogue=L.EPI_ATOMIC, split_k=F._split_k(3072, 768, T), prec=p, colsum=dbi)),
 "bert_ffn2_wgrad_cs": (2*T*768*3072, lambda p: K.gemm(768, 3072, T, K.operand(o, L.MNCONTIG), K.operand(G, L.MNCONTIG), dWo2, epilogue=L.EPI_ATOMIC, split_k=F._split_k(768, 3072, T), prec=p, colsum=dbo2)),
 "bert_qkv_wgrad_cs": (2*T*768*2304, lambda p: K.gemm(2304, 768, T, K.operand(qkv, L.MNCONTIG), K.operand(x, L.MNCONTIG), dWqkv, epilogue=L.EPI_ATOMIC, split_k=F._split_k(2304, 768, T), prec=p, colsum=dbqkv)),
 "bert_ffn2_dgrad": (2*T*768*3072, lambda p: K.gemm(T, 3072, 768, K.operand(o, L.KCONTIG), K.operand(wo2, L.MNCONTIG), Ub, prec=p)),
 "bert_qkv_dgrad": (2*T*768*2304, lambda p: K.gemm(T, 768, 2304, K.operand(qkv, L.KCONTIG), K.operand(wqkv, L.MNCONTIG), x, prec=p)),
 "bert_ffn1_wgrad_atomic": (2*T*768*3072, lambda p: L.call("nr_gemm_f32", 3072, 768, T, K.operand(G, L.MNCONTIG), K.operand(x, L.MNCONTIG), L.ptr(dWi), 768, None, L.EPI_ATOMIC, None, -1, F._split_k(3072, 768, T), p, L.stream_ptr(dWi))),
 "cnn_conv_wgrad": (2*U*E*480, lambda p: K.gemm_dyn(480, E, U, K.operand(Pg, L.MNCONTIG), K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_GATHER), dw3, epilogue=L.EPI_ATOMIC, split_k=F._split_k(480, E, U), prec=p)),
 "cnn_table_dgrad_kc": (2*24600*E*480, lambda p: K.gemm_dyn(U, E, 480, K.operand(Pg, L.KCONTIG), K.operand(w3T, L.KCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p)),
 "cnn_table_dgrad": (2*24600*E*480, lambda p: K.gemm_dyn(U, E, 480, K.operand(Pg, L.KCONTIG), K.operand(w3, L.MNCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p)),
 "nrms_dgrad_table_kc_ws": (2*24600*E*1152, lambda p: K.gemm_dyn(52800, E, 1152, K.operand(dYc, L.KCONTIG), K.operand(WT, L.KCONTIG), dT, m_dev=m_dev, epilogue=L.EPI_SCATTER_ZEROED, c_rows=K.rows_map(uids, L.ROWS_GATHER), pad_row=0, prec=p, workspace=True)),
 "nrms_proj_wgrad_atomic": (2*U*E*1152, lambda p: L.call("nr_gemm_f32_dyn", 1152, E, U, K.operand(dY, L.MNCONTIG), K.operand(table, L.MNCONTIG, rows=ids, mapping=L.ROWS_GATHER), L.ptr(dW), E, None, L.EPI_ATOMIC, None, -1, F._split_k(1152, E, U), None, None, p, L.stream_ptr(dW))),
}
out = {}
import os
only = os.environ.get("NR_AB_CASES")
for pn, p in (("bf16x6", L.GEMM_BF16X6), ("bf16", L.GEMM_BF16)):
    for k, (fl, fn) in cases.items():
        if only and k not in only.split(","):
            continue
        ms = bench(lambda: fn(p))
        out.setdefault(k, {})[pn] = {"us": round(ms * 1e3, 1), "tflops": round(fl / ms / 1e9, 1)}
print(json.dumps(out))
''' % ROOT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="base",
                    help="comma-separated library paths ('base' = the in-tree build)")
    ap.add_argument("--cases", default=None, help="comma-separated case names (default: all)")
    a = ap.parse_args()
    res = {}
    for m in a.libs.split(","):
        env = dict(os.environ)
        env.pop("NR_LIB_PATH", None)
        if m != "base":
            env["NR_LIB_PATH"] = os.path.abspath(m)
        if a.cases:
            env["NR_AB_CASES"] = a.cases
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            res[m] = {"error": r.stderr[-2000:]}
            print(json.dumps({m: res[m]}), flush=True)
            break
        key = m if m not in res else "%s#%d" % (m, len(res))
        res[key] = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps({key: res[key]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
