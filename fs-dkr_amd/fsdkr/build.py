"""Builds libfsdkr.so (gfx950 HIP kernels + C ABI) in-tree with hipcc.

Objects go to fs-dkr_amd/build/, the shared library to
fs-dkr_amd/fsdkr/libfsdkr.so (git-ignored, but shipped to the GPU box by
gpurun).  Incremental on source/header mtimes."""
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                 # fs-dkr_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libfsdkr.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["modexp.hip", "verify.hip", "inverse.hip", "capi.cpp", "collect.cpp", "recover.cpp", "standalone.cpp"]
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
          "-Wno-unused-result"]


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hpp"))]
    hs += [os.path.join(INCLUDE, "fsdkr", f) for f in os.listdir(os.path.join(INCLUDE, "fsdkr"))]
    return hs


def _compile(src, verbose):
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC] + CFLAGS + ["-c", os.path.join(CSRC, src), "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False, force=False):
    os.makedirs(BUILD, exist_ok=True)
    hdr_mtime = max(os.path.getmtime(h) for h in _headers())
    todo, objs = [], []
    for src in SOURCES:
        obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        stale = force or not os.path.exists(obj) or \
            os.path.getmtime(obj) < max(os.path.getmtime(os.path.join(CSRC, src)), hdr_mtime)
        if stale:
            todo.append(src)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(todo))) as ex:
            list(ex.map(lambda s: _compile(s, verbose), todo))
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
