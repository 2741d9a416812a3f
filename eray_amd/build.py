"""Build recipe of the product library eray_amd/lib/liberay_hip.so (gfx950 only).

    python -m eray_amd.build [--jobs N] [--verbose]

Compiles the HIP kernels and the C-ABI layer with hipcc for gfx950 and links them into one
shared library next to this package, so it travels to the GPU box with the repository.
Floating-point flags are part of the contract: -ffp-contract=off keeps a*b+c unfused so the
kernels reproduce the reference's f32 results bit-for-bit; hipcc's defaults already give
correctly rounded f32 division/sqrt and keep f32 denormals.
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
OBJ = os.path.join(PKG, "_obj")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "liberay_hip.so")

SOURCES = ["render.hip", "setup.hip", "trace.hip", "bins.hip", "shaderlib.hip", "capi.cpp", "comm.cpp", "objload.cpp"]
ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
            f"--offload-arch={ARCH}", "-I" + os.path.join(ROOT, "include"),
            # the first 15 kernel-argument dwords arrive in SGPRs (frame_kernel's FrameHot + band word)
            "-mllvm", "-amdgpu-kernarg-preload-count=15"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the eray_amd HIP library cannot be built")


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _headers() -> list[str]:
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    hs.append(os.path.join(ROOT, "include", "eray_hip.h"))
    return hs


def build(jobs: int = 4, verbose: bool = False, force: bool = False) -> str:
    """Build the product library (the only build: no diagnostic variants of the kernels)."""
    obj_dir = OBJ
    lib_path = LIB
    extra: list[str] = []
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    cc = hipcc()
    headers = _headers()
    objs, cmds = [], []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(obj_dir, src + ".o")
        objs.append(o)
        if force or not _newer(o, [s] + headers):
            lang = [] if src.endswith(".hip") else ["-x", "hip"]
            cmds.append([cc, *CXXFLAGS, *extra, *lang, "-c", s, "-o", o])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return r.stderr

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for warn in ex.map(run, cmds):
            if warn.strip() and verbose:
                print(warn, file=sys.stderr)
    if force or cmds or not _newer(lib_path, objs):
        # RCCL for the multi-GPU gather (comm.cpp); under PyTorch the loader reuses torch's copy
        # (same SONAME librccl.so.1), so one RCCL serves the process
        run([cc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path, *objs, "-L/opt/rocm/lib", "-lrccl",
             "-Wl,-rpath,/opt/rocm/lib"])
    return lib_path


HOST_SOURCES = ["image.cpp", "graph.cpp", "shaderlib.cpp", "engine.cpp"]
HOST_LIB = os.path.join(LIB_DIR, "liberay_host.so")
BIN_DIR = os.path.join(PKG, "bin")
ROCM_LIB = "/opt/rocm/lib"


def build_host(jobs: int = 4, verbose: bool = False, force: bool = False) -> list[str]:
    """The C++ host (include/eray/, eray_amd/host/): liberay_host.so over the C-ABI library,
    the eray_main CLI (main.rs) and the tests/cpp/test_host unit-test binary.  Plain g++: the
    host code never includes HIP headers."""
    hip_lib = build(jobs, verbose, force)
    host = os.path.join(PKG, "host")
    cxx = shutil.which("g++") or "g++"
    flags = ["-std=c++17", "-O2", "-fPIC", "-Wall", "-I" + os.path.join(ROOT, "include")]
    headers = [os.path.join(ROOT, "include", "eray", f) for f in os.listdir(os.path.join(ROOT, "include", "eray"))]
    headers.append(os.path.join(ROOT, "include", "eray_hip.h"))
    obj_dir = os.path.join(OBJ, "host")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(BIN_DIR, exist_ok=True)
    link = ["-L" + LIB_DIR, "-leray_hip", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,$ORIGIN/../lib",
            "-Wl,-rpath-link," + ROCM_LIB, "-Wl,-rpath," + ROCM_LIB]

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"host build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")

    objs, cmds = [], []
    for src in HOST_SOURCES:
        s, o = os.path.join(host, src), os.path.join(obj_dir, src + ".o")
        objs.append(o)
        if force or not _newer(o, [s] + headers):
            cmds.append([cxx, *flags, "-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(run, cmds))
    if force or cmds or not _newer(HOST_LIB, objs + [hip_lib]):
        run([cxx, "-shared", "-o", HOST_LIB, *objs, *link])
    outs = [HOST_LIB]
    for name, src in (("eray_main", os.path.join(host, "main.cpp")),
                      ("test_host", os.path.join(ROOT, "tests", "cpp", "test_host.cpp"))):
        exe = os.path.join(BIN_DIR, name)
        if force or not _newer(exe, [src, HOST_LIB] + headers):
            run([cxx, *flags, src, "-o", exe, "-L" + LIB_DIR, "-leray_host", *link])
        outs.append(exe)
    return outs


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--host", action="store_true", help="also build the C++ host (liberay_host.so, bin/)")
    a = ap.parse_args()
    print(build(a.jobs, a.verbose, a.force))
    if a.host:
        print("\n".join(build_host(a.jobs, a.verbose, a.force)))


if __name__ == "__main__":
    main()
