#!/usr/bin/env python3
"""Build the native extension `apex_example_amd/_C*.so` for gfx950, in-tree.

No hipify, no torch JIT cache: HIP kernels (csrc/hip/*.hip) are compiled with
`hipcc --offload-arch=gfx950` and never include torch headers; the torch-facing
C++ (csrc/torch/*.cpp, csrc/cpu/*.cpp) is compiled with g++ against the torch
headers and linked with the kernels into one shared object that loads on CPU-only
hosts too (the CPU paths are plain C++).

Incremental: an object is rebuilt when its source or any header under csrc/ is
newer than it.  Objects go to build/obj/.

    python tools/build_ext.py [-j N] [--clean] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
PKG = os.path.join(ROOT, "apex_example_amd")
ARCH = os.environ.get("APEX_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch  # noqa: F401
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, lib


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _sources():
    hip, cpp = [], []
    for sub in ("hip",):
        d = os.path.join(CSRC, sub)
        hip += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".hip"))
    for sub in ("torch", "cpu"):
        d = os.path.join(CSRC, sub)
        cpp += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".cpp"))
    return hip, cpp


def _newest_header() -> float:
    t = 0.0
    for dp, _, fs in os.walk(CSRC):
        for f in fs:
            if f.endswith((".h", ".hpp", ".cuh")):
                t = max(t, os.path.getmtime(os.path.join(dp, f)))
    return t


def _obj_for(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(OBJ, rel + ".o")


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    t0 = time.time()
    p = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if p.returncode != 0:
        raise RuntimeError("command failed (%d):\n%s\n%s" % (p.returncode, " ".join(cmd), p.stdout))
    return time.time() - t0, p.stdout


def build(jobs: int | None = None, verbose: bool = False, clean: bool = False) -> str:
    if clean and os.path.isdir(OBJ):
        shutil.rmtree(OBJ)
    os.makedirs(OBJ, exist_ok=True)
    tinc, tlib = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    hdr_t = _newest_header()
    hip_srcs, cpp_srcs = _sources()
    inc_flags = ["-I" + os.path.join(CSRC, "include")]

    hip_cmd = lambda s, o: [  # noqa: E731
        os.path.join(ROCM, "bin", "hipcc"), "-c", "-O3", "-std=c++17", "-fPIC",
        "--offload-arch=" + ARCH, "-D__HIP_PLATFORM_AMD__=1", "-munsafe-fp-atomics",
        "-Wno-unused-result", *inc_flags, s, "-o", o,
    ]
    cxx = os.environ.get("CXX", "g++")
    cpp_cmd = lambda s, o: [  # noqa: E731
        cxx, "-c", "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-deprecated-declarations", *inc_flags,
        *["-I" + p for p in tinc], "-I" + py_inc, s, "-o", o,
    ]

    todo = []
    objs = []
    for s in hip_srcs + cpp_srcs:
        o = _obj_for(s)
        objs.append(o)
        if (not os.path.exists(o)) or os.path.getmtime(o) < max(os.path.getmtime(s), hdr_t):
            todo.append((s, o, hip_cmd(s, o) if s.endswith(".hip") else cpp_cmd(s, o)))

    jobs = jobs or min(8, os.cpu_count() or 4)
    t0 = time.time()
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_run, c, verbose): s for s, _, c in todo}
            for f in cf.as_completed(futs):
                dt, _ = f.result()
                print("  [%5.1fs] %s" % (dt, os.path.relpath(futs[f], ROOT)), flush=True)
    out = ext_path()
    if todo or not os.path.exists(out):
        link = [
            os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", "--offload-arch=" + ARCH,
            *objs, "-o", out, "-L" + tlib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-ltorch_python", "-lhipblaslt", "-lroctx64", "-Wl,-rpath," + tlib,
        ]
        _run(link, verbose)
        # an unresolved symbol only shows at dlopen: check the fresh .so in a child
        chk = subprocess.run([sys.executable, "-c", "import torch, importlib.util as u; "
                              "s = u.spec_from_file_location('_C', %r); "
                              "u.module_from_spec(s)" % out],
                             capture_output=True, text=True)
        if chk.returncode != 0:
            os.remove(out)
            raise RuntimeError("built extension does not load:\n" + chk.stderr[-2000:])
    print("built %s (%d objects rebuilt, %.1fs)" % (os.path.relpath(out, ROOT), len(todo),
                                                   time.time() - t0), flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    build(a.jobs, a.verbose, a.clean)


if __name__ == "__main__":
    sys.exit(main())
