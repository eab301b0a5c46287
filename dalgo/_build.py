"""In-tree native build of the dalgo HIP extension (gfx950 only).

Compiles every ``csrc/kernels/*.hip`` with ``hipcc --offload-arch=gfx950`` (pure
HIP, no torch headers: fast, cacheable), the torch-op registration layer
``csrc/bindings.cpp`` with the host C++ compiler against the torch headers,
and links them into ``dalgo/_dalgo_hip.so``. The shared object stays in-tree so
it travels with the repository snapshot to the GPU box (a JIT cache under
``~/.cache`` would not).

Usage: ``python -m dalgo._build [--force] [-j N]``; ``__graft_entry__.build()``
calls :func:`build`.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
OUT = ROOT / "dalgo" / "_dalgo_hip.so"
ARCH = "gfx950"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return p


def _torch_paths():
    import torch  # noqa: F401  (only for its install location)
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    return tdir, inc, tdir / "lib"


def _cxx11_abi() -> int:
    import torch
    return int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newest(paths) -> float:
    m = 0.0
    for p in paths:
        try:
            m = max(m, p.stat().st_mtime)
        except FileNotFoundError:
            pass
    return m


def _run(cmd, verbose):
    if verbose:
        print(" ".join(map(str, cmd)), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n$ {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


def kernel_sources():
    return sorted((CSRC / "kernels").glob("*.hip"))


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Build (incrementally) and return the path of ``_dalgo_hip.so``."""
    BUILD.mkdir(parents=True, exist_ok=True)
    headers = list((CSRC / "include").rglob("*.h")) + [CSRC / "launchers.h"]
    hdr_time = _newest(headers)
    hipcc = _hipcc()
    jobs = jobs or min(8, os.cpu_count() or 4)

    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC / 'include'}", f"-I{CSRC}"]
    jobs_list = []
    objs = []
    for src in kernel_sources():
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_time):
            jobs_list.append([hipcc, f"--offload-arch={ARCH}", *common, "-munsafe-fp-atomics",
                              "-c", src, "-o", obj])

    tdir, tinc, tlib = _torch_paths()
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    objs.append(bobj)
    if force or not bobj.exists() or bobj.stat().st_mtime < max(bsrc.stat().st_mtime, hdr_time):
        cxx = os.environ.get("CXX", "g++")
        pyinc = sysconfig.get_paths()["include"]
        jobs_list.append([cxx, "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1",
                          "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={_cxx11_abi()}",
                          *[f"-I{p}" for p in tinc], f"-I{ROCM / 'include'}", f"-I{pyinc}",
                          f"-I{CSRC}", "-Wno-deprecated-declarations", "-c", bsrc, "-o", bobj])

    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))

    if force or not OUT.exists() or OUT.stat().st_mtime < _newest(objs):
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", OUT,
              f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
              f"-Wl,-rpath,{tlib}", f"-L{ROCM / 'lib'}", "-lamdhip64",
              "-Wl,--no-undefined"], verbose)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    out = build(force=a.force, jobs=a.jobs, verbose=a.verbose)
    print(f"built {out}")


if __name__ == "__main__":
    sys.exit(main())
