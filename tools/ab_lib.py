#!/usr/bin/env python3
"""A/B of a library built from a previous revision of one source: compile `src_file` (a
copy of e.g. csrc/prover.cpp from an older commit) with the current build's flags and link
it with the other objects of the current build into lib_ab/libh2g_<tag>.so.
usage: python tools/ab_lib.py TAG SRC_FILE OBJ_TO_REPLACE   (e.g. prev /tmp/prover.cpp prover.cpp)"""
import glob
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "yet-another-halo2-fork_amd"))
import build_lib as B  # noqa: E402

tag, src, replaced = sys.argv[1:4]
out_dir = os.path.join(B.PKG, "lib_ab")
os.makedirs(out_dir, exist_ok=True)
objs = [o for o in glob.glob(os.path.join(B.BUILD, "*.o")) if not o.endswith(replaced + ".o")]
obj = os.path.join(out_dir, f"{tag}.o")
subprocess.run([B.HIPCC] + B.CFLAGS + ["-I", B.CSRC, "-x", "hip", "-c", src, "-o", obj], check=True)
lib = os.path.join(out_dir, f"libh2g_{tag}.so")
subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", lib] + objs + [obj] +
               ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"], check=True)
print(lib)
