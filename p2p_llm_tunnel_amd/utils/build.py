"""Build helpers for the native core (CMake + Ninja) and the HIP kernels."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

from p2p_llm_tunnel_amd import BIN_DIR, PKG_DIR, REPO_ROOT

BUILD_DIR = os.path.join(REPO_ROOT, "build")


def _newest_mtime(paths) -> float:
    newest = 0.0
    for root in paths:
        for dp, _, files in os.walk(root):
            for f in files:
                if f.endswith((".cc", ".h", ".txt")):
                    newest = max(newest, os.path.getmtime(os.path.join(dp, f)))
    return newest


def native_outputs() -> list[str]:
    import glob
    outs = [os.path.join(BIN_DIR, n) for n in ("tunnel", "tunnel-signal", "tunnel-mock", "tunnel-loadgen",
                                                "native_tests")]
    outs += glob.glob(os.path.join(PKG_DIR, "_native*.so"))
    return outs


def native_up_to_date() -> bool:
    outs = native_outputs()
    if len(outs) < 6 or not all(os.path.exists(o) for o in outs):
        return False
    src = _newest_mtime([os.path.join(REPO_ROOT, "native")])
    src = max(src, os.path.getmtime(os.path.join(REPO_ROOT, "CMakeLists.txt")))
    return min(os.path.getmtime(o) for o in outs) >= src


def build_native(jobs: int | None = None, quiet: bool = True, build_type: str = "Release") -> None:
    """Configure (once) and build the C++ core: tunnel, tunnel-signal, native_tests, _native."""
    jobs = jobs or min(16, os.cpu_count() or 4)
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    out = subprocess.DEVNULL if quiet else None
    if not os.path.exists(os.path.join(BUILD_DIR, "CMakeCache.txt")):
        subprocess.run(["cmake", "-S", REPO_ROOT, "-B", BUILD_DIR, *gen, f"-DCMAKE_BUILD_TYPE={build_type}",
                        f"-DPython3_EXECUTABLE={sys.executable}"], check=True, stdout=out)
    r = subprocess.run(["cmake", "--build", BUILD_DIR, "-j", str(jobs)], stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("native build failed:\n" + r.stdout[-8000:])


def ensure_native() -> None:
    if not native_up_to_date():
        build_native()
