"""Compile the HIP kernels in-tree for gfx950 (CDNA4 / MI355X).

    hipcc -O3 --offload-arch=gfx950 -shared -fPIC kernels.hip decode_fused.hip sample.hip -o _hip_ops.so

Cross-compiles on a CPU-only host; the .so travels with the repo snapshot to
the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, f) for f in ("kernels.hip", "decode_fused.hip", "sample.hip")]
DEPS = SRCS + [os.path.join(HERE, "bf16_common.h")]
OUT = os.path.join(HERE, "_hip_ops.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def up_to_date() -> bool:
    return os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in DEPS)


def build(verbose: bool = False, force: bool = False) -> str:
    if up_to_date() and not force:
        return OUT
    cmd = [hipcc(), "-O3", f"--offload-arch={ARCH}", "-std=c++17", "-shared", "-fPIC", "-o", OUT + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stdout[-8000:])
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(verbose=True, force=True))
