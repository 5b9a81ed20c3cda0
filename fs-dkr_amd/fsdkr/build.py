"""Builds libfsdkr.so (gfx950 HIP kernels + C ABI) in-tree with hipcc.

Objects go to fs-dkr_amd/build/, the shared library to
fs-dkr_amd/fsdkr/libfsdkr.so (git-ignored, but shipped to the GPU box by
gpurun).  Incremental: each object is rebuilt when its source or any header it
includes (hipcc -MMD dependency file) is newer."""
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

SOURCES = ["modexp.hip", "fixedbase.hip", "comb.hip", "inverse.hip", "vhash.hip", "vmont.hip", "vec.hip", "pow2.hip",
           "prime.hip", "capi.cpp", "keygen.cpp", "collect.cpp", "collect_prestart.cpp", "collect_prepare.cpp",
           "collect_launch.cpp", "recover.cpp", "standalone.cpp", "fixedbase_host.cpp"]
CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
          "-Wno-unused-result"]


def _obj(src):
    return os.path.join(BUILD, os.path.splitext(src)[0] + ".o")


def _deps(src):
    """Files the object depends on, from the -MMD file of its last build."""
    dep = _obj(src)[:-2] + ".d"
    if not os.path.exists(dep):
        return None
    text = open(dep).read().replace("\\\n", " ")
    files = text.split(":", 1)[1].split() if ":" in text else []
    return [f for f in files if f.endswith((".h", ".hpp", ".hip", ".cpp"))]


def _stale(src, force):
    obj = _obj(src)
    if force or not os.path.exists(obj):
        return True
    deps = _deps(src)
    if deps is None:
        return True
    t = os.path.getmtime(obj)
    return any(not os.path.exists(f) or os.path.getmtime(f) > t for f in deps + [os.path.join(CSRC, src)])


def _compile(src, verbose):
    obj = _obj(src)
    cmd = [HIPCC] + CFLAGS + ["-MMD", "-MF", obj[:-2] + ".d", "-c", os.path.join(CSRC, src), "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def _build_pack(verbose):
    """The CPython extension of the batching layer (csrc/pack.c -> fsdkr/_pack*.so)."""
    import sysconfig
    src = os.path.join(CSRC, "pack.c")
    out = os.path.join(PKG, "_pack" + sysconfig.get_config_var("EXT_SUFFIX"))
    if os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(src):
        return out
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-I", sysconfig.get_paths()["include"], src, "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"pack extension build failed:\n{r.stdout}\n{r.stderr}")
    return out


def build(verbose=False, force=False):
    os.makedirs(BUILD, exist_ok=True)
    _build_pack(verbose)
    todo = [s for s in SOURCES if _stale(s, force)]
    objs = [_obj(s) for s in SOURCES]
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(8, len(todo))) as ex:
            list(ex.map(lambda s: _compile(s, verbose), todo))
    if todo or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lcrypto"]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
