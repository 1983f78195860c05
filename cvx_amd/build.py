"""Build libcvxg.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo snapshot)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcvxg.so")
SOURCES = ["k_vec.hip", "k_syrk.hip", "k_chol.hip", "k_dataflow.hip", "k_ruiz.hip", "k_pd.hip", "k_quad.hip", "symsolve.cpp", "affine.cpp", "k_kkt.hip", "cvxg.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "cvxg.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    # -ffp-contract=off: every a*b+c is rounded twice unless the source says fma(), so the elementwise steps the
    # reference evaluates as separate Breeze operations (x + s*t, d*d, t*(a + Px) + ...) keep its roundings;
    # the dot products and MFMA accumulations use explicit fma / MFMA builtins.
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall",
           "-Wno-pass-failed", "-Wl,-z,defs", "-o", OUT + ".tmp"] + [os.path.join(CSRC, s) for s in SOURCES] + [
        "-L/opt/rocm/lib", "-lrocsolver", "-lrocblas", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
