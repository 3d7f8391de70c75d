"""Build libi2pc.so (all HIP kernels + the C ABI) for gfx950, in-tree.

    python -m image_to_pointcloud_amd.build [-j N] [--force]

Each source compiles to its own object under build/ (hipcc cross-compiles for
gfx950 without a GPU) and the objects link into
image_to_pointcloud_amd/libi2pc.so, which travels to the GPU box with the repo
snapshot.  Rebuilds only sources newer than their object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(ROOT, "build", "i2pc")
LIB = os.path.join(PKG, "libi2pc.so")
ARCH = os.environ.get("I2PC_ARCH", "gfx950")

SOURCES = [
    "abi.cpp",
    "unproject.hip",
    "gemm.hip",
    "misc.hip",
    "attention.hip",
    "preprocess.hip",
    "sor.hip",
    "head.hip",
    "area.hip",
    "fp8.hip",
    "bit.hip",
    "probe.hip",
    "model.cpp",
    "comm.cpp",
    "writers.cpp",
]
HEADERS = ["common.h", "mx.h", "../../include/i2pc.h"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libi2pc.so)")


def _flags(src: str) -> list[str]:
    f = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-I", os.path.join(ROOT, "include")]
    if src.endswith(".cpp"):
        f = ["-x", "hip"] + f
    return f


def _newest_header() -> float:
    return max(os.path.getmtime(os.path.join(CSRC, h)) for h in HEADERS)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    path = os.path.join(CSRC, src)
    if (not force and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(path), _newest_header())):
        return obj
    cmd = [hipcc()] + _flags(src) + ["-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if (force or not os.path.exists(LIB)
            or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs)):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lrccl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    _build_example(force)
    if verbose:
        print(f"built {LIB}")
    return LIB


EXAMPLE = os.path.join(ROOT, "examples", "depth_forward")


def _build_example(force: bool) -> None:
    """examples/depth_forward: a plain C caller of the network executor (gcc, HIP's C API, libi2pc.so)."""
    src = EXAMPLE + ".c"
    if not os.path.exists(src):
        return
    if (not force and os.path.exists(EXAMPLE)
            and os.path.getmtime(EXAMPLE) >= max(os.path.getmtime(src), os.path.getmtime(LIB))):
        return
    rocm = os.path.dirname(os.path.dirname(os.path.realpath(hipcc())))
    cmd = [shutil.which("gcc") or "gcc", "-std=c99", "-O2", "-Wall", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(rocm, "include"), "-I", os.path.join(ROOT, "include"), src, "-o", EXAMPLE,
           "-L", PKG, "-li2pc", "-L", os.path.join(rocm, "lib"), "-lamdhip64",
           "-Wl,-rpath,$ORIGIN/../image_to_pointcloud_amd", "-Wl,-rpath," + os.path.join(rocm, "lib")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"example build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    build(a.jobs, a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
