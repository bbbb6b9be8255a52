"""Build libnewsrec_hip.so for gfx950 in-tree (the .so travels to the GPU box with the
snapshot).  Every csrc/*.hip is compiled to an object in parallel, then linked against
libamdhip64 only — the library has no torch dependency (C ABI in include/newsrec_hip.h).

Provenance: the library embeds a hash of every source it is built from (csrc/*.hip, csrc/*.h,
include/*.h and the compiler flags), returned by nr_build_hash().  Objects are cached under a name
that carries the hash of their own inputs (never by mtime), the link is redone whenever the source
hash changes, and newsrec_amd._lib refuses to load a library whose hash differs from the sources
next to it — a GPU run provably uses the kernels of the tree it was sent with.
"""
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
OUT = os.path.join(HERE, "newsrec_amd", "lib")
LIB = os.path.join(OUT, "libnewsrec_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics", "-I" + INCLUDE]
# Per-source flags.  The bf16x6 GEMM units build without SLP vectorisation: it packs the operand
# split's f32 subtractions (and the loaders' selects / column-sum adds) into v_pk_add_f32, and packed
# f32 VALU beside MFMAs costs ≈ +11 cycles per instruction over its scalar pair (MI355X_MICROARCH.md,
# cycle constants).  One-box A/B (tools/gemm_ab.py, bf16x6): projection fwd 295 -> 258 µs, table dgrad
# 309 -> 301, weight gradient 348 -> 300, BERT FFN weight gradient 583 -> 409.  The bf16 (one-plane)
# units keep it: there it measured neutral to 12 % slower.
EXTRA = {name: ["-fno-slp-vectorize"] for name in
         ("gemm_big_3_256.hip", "gemm_big_3_128.hip", "gemm_split_kc3.hip", "gemm_split_mn3.hip")}


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))


def source_hash():
    """16 hex digits over the library's sources, headers and flags (what nr_build_hash returns)."""
    h = hashlib.sha256()
    for p in _sources() + _headers():
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(_flags_key())
    h.update(repr(sorted(EXTRA.items())).encode())
    return h.hexdigest()[:16]


def _flags_key():
    """The compiler flags without the checkout's absolute paths (the hash must not depend on where
    the tree lives: the GPU box unpacks it elsewhere)."""
    return " ".join(f if not f.startswith("-I") else "-I<include>" for f in FLAGS).encode()


def _obj_name(src, hdr_digest):
    h = hashlib.sha256()
    with open(src, "rb") as f:
        h.update(f.read())
    h.update(hdr_digest.encode())
    h.update(" ".join(EXTRA.get(os.path.basename(src), [])).encode())
    return os.path.join(OUT, "obj", "%s.%s.o" % (os.path.basename(src), h.hexdigest()[:12]))


def _compile(job):
    src, obj, extra = job
    if os.path.exists(obj):
        return obj
    tmp = obj + ".tmp%d" % os.getpid()
    cmd = [HIPCC] + FLAGS + extra + ["-c", src, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed on %s:\n%s" % (src, r.stderr[-6000:]))
    os.replace(tmp, obj)
    return obj


def _write_version(digest):
    """The one translation unit that carries the source hash."""
    path = os.path.join(OUT, "obj", "version.cpp")
    text = ('extern "C" const char* nr_build_hash(void) { return "%s"; }\n' % digest)
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(verbose=True):
    os.makedirs(os.path.join(OUT, "obj"), exist_ok=True)
    digest = source_hash()
    hdr = hashlib.sha256()
    for p in _headers():
        with open(p, "rb") as f:
            hdr.update(f.read())
    hdr.update(_flags_key())
    hdr_digest = hdr.hexdigest()
    jobs = [(s, _obj_name(s, hdr_digest), EXTRA.get(os.path.basename(s), [])) for s in _sources()]
    workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(_compile, jobs))
    stamp = os.path.join(OUT, "obj", "lib.hash")
    have = open(stamp).read().strip() if os.path.exists(stamp) else None
    if not os.path.exists(LIB) or have != digest:
        ver = _write_version(digest)
        ver_obj = os.path.join(OUT, "obj", "version.o")
        r = subprocess.run(["g++", "-fPIC", "-O2", "-c", ver, "-o", ver_obj], capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("version object failed:\n" + r.stderr[-2000:])
        tmp = LIB + ".tmp%d" % os.getpid()
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs + [ver_obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stderr[-4000:])
        os.replace(tmp, LIB)
        with open(stamp, "w") as f:
            f.write(digest)
    # drop cached objects of older sources
    keep = set(objs)
    for o in glob.glob(os.path.join(OUT, "obj", "*.hip.*.o")):
        if o not in keep:
            os.remove(o)
    if verbose:
        print("built", LIB, "source hash", digest)
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
