#!/usr/bin/env python3
"""Build libh2g.so (HIP kernels + C ABI) for gfx950, in tree.

    python yet-another-halo2-fork_amd/build_lib.py [--force]

Objects go to yet-another-halo2-fork_amd/build/, the library to
yet-another-halo2-fork_amd/lib/libh2g.so (git-ignored; travels to the GPU box
with the gpurun snapshot).  Incremental: a source is recompiled when it or a header it
includes (transitively) is newer than its object.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "build")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libh2g.so")
ARCH = os.environ.get("H2G_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-I", CSRC, "-I", os.path.join(os.path.dirname(PKG), "include")]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


INC_DIRS = (CSRC, os.path.join(os.path.dirname(PKG), "include"))


def _includes(path, seen):
    """the quoted includes of `path`, transitively (csrc/ and include/)"""
    for line in open(path, errors="replace"):
        line = line.strip()
        if not line.startswith("#include \""):
            continue
        name = line.split('"')[1]
        for d in INC_DIRS:
            h = os.path.join(d, name)
            if os.path.exists(h) and h not in seen:
                seen.add(h)
                _includes(h, seen)
                break
    return seen


def _newest_dep(src):
    return max((os.path.getmtime(h) for h in _includes(src, set())), default=0)


def compile_one(src, force):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if not force and os.path.exists(obj):
        t = os.path.getmtime(obj)
        if t >= os.path.getmtime(src) and t >= _newest_dep(src):
            return obj, None
    lang = ["-x", "hip"] if src.endswith(".hip") else ["-x", "hip"]
    cmd = [HIPCC] + CFLAGS + lang + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, len(srcs))
    objs, errs = [], []
    with cf.ThreadPoolExecutor(jobs) as ex:
        for obj, err in ex.map(lambda s: compile_one(s, force), srcs):
            objs.append(obj)
            if err:
                errs.append(err)
    if errs:
        raise RuntimeError("libh2g build failed:\n" + "\n".join(errs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + [
            "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
