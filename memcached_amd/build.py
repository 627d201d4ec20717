"""Build the native pieces in-tree (no JIT cache, so the .so files travel to
the GPU box with the repository snapshot).

    python -m memcached_amd.build          # libmcrc32c.so (+ oracle/ test libs)

libmcrc32c.so: crc32c_shim.hip (+ the kernels it includes) compiled by hipcc for
gfx950, linked with the host CRC (crc32c_host.cpp, g++ -O2).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libmcrc32c.so")
ARCH = os.environ.get("MCRC_ARCH", "gfx950")


def _run(cmd, cwd=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=cwd)


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def build_lib(force: bool = False) -> str:
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps += [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))]
    if not force and _newer(LIB, deps):
        return LIB
    tmp = os.path.join(CSRC, "_obj")
    os.makedirs(tmp, exist_ok=True)
    host_o = os.path.join(tmp, "crc32c_host.o")
    shim_o = os.path.join(tmp, "crc32c_shim.o")
    _run(["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-c", os.path.join(CSRC, "crc32c_host.cpp"),
          "-o", host_o])
    _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
          os.path.join(CSRC, "crc32c_shim.hip"), "-o", shim_o])
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, shim_o, host_o,
          "-lpthread"])
    shutil.rmtree(tmp, ignore_errors=True)
    return LIB


def build_oracle() -> None:
    """Test infrastructure (oracle/Makefile): the CPU restatement and, when
    /root/reference exists (build container only), the reference build."""
    _run(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


def build_all(force: bool = False) -> None:
    build_lib(force)
    build_oracle()


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
