"""A/B build: libh2g with one source (default msm.hip) compiled under extra -D flags,
linked with the other objects of the current build into
yet-another-halo2-fork_amd/lib_ab/libh2g_<tag>.so (select it with H2G_LIB).
usage: python tools/build_variant.py TAG [--src msm_acc.hip[,msm_part.hip]] -DNAME=VALUE ..."""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))
import build_lib as B  # noqa: E402

tag, defs = sys.argv[1], sys.argv[2:]
names = ["msm.hip"]
if defs[:1] == ["--src"]:  # one source or several, comma separated
    names, defs = defs[1].split(","), defs[2:]
B.build()
out_dir = os.path.join(B.PKG, "lib_ab")
os.makedirs(out_dir, exist_ok=True)
objs = [o for o in glob.glob(os.path.join(B.BUILD, "*.o")) if not any(o.endswith(nm + ".o") for nm in names)]
for name in names:
    obj = os.path.join(out_dir, f"{name.split('.')[0]}_{tag}.o")
    src = os.path.join(B.CSRC, name)
    subprocess.run([B.HIPCC] + B.CFLAGS + defs + ["-x", "hip", "-c", src, "-o", obj], check=True)
    objs.append(obj)
lib = os.path.join(out_dir, f"libh2g_{tag}.so")
subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", lib] + objs +
               ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
print(lib)
