#!/usr/bin/env python3
"""In-tree native build for ntxent-mi355x (gfx950 only).

Drives hipcc directly — no hipify pass, no torch JIT cache — and drops the extension
next to the Python package so it travels with the repo snapshot to the GPU box:

  <pkg>/_C.<abi>.so            PyTorch extension (pybind11 + TORCH_LIBRARY)
  build/bin/ntxent_bench       C++ benchmark (reference src/benchmark.cpp)
  build/bin/ntxent_tests       C++ tests    (reference tests/test_*.cpp)

Incremental: an object is rebuilt only when a source or header it depends on is newer.
Usage: python tools/build_ext.py [--force] [--no-cpp] [-v]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "cuda-nt-xent-mpi-nccl-simclr_amd"
CSRC = PKG / "csrc"
BUILD = ROOT / "build"
ARCH = os.environ.get("NTXENT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


RUNTIME_SRCS = ["engine.cpp", "engine_sym.cpp", "rccl_comm.cpp", "trace.cpp"]
KERNEL_SRCS = [CSRC / "kernels" / "ntxent_kernels.hip", CSRC / "kernels" / "small_kernels.hip"]


def _host_cxx():
    """hipcc as a plain host C++ compiler (no device pass) for runtime / torch / tool TUs."""
    return [HIPCC, "-x", "c++", "-D__HIP_PLATFORM_AMD__=1", "-std=c++17", "-fPIC", "-I/opt/rocm/include"]


def _feature_defines():
    """Compile-time feature switches (mirrors the CMake options)."""
    d = []
    if os.environ.get("NTXENT_ENABLE_PROFILING", "0") == "1":
        d.append("-DNTXENT_PROFILING_DEFAULT=1")
    if os.environ.get("NTXENT_USE_FP16", "1") == "0":  # CMake USE_FP16=OFF
        d.append("-DNTXENT_DEFAULT_COMPUTE_BF16=1")
    if os.environ.get("NTXENT_ENABLE_FP8", "1") == "0":  # CMake ENABLE_FP8=OFF
        d.append("-DNTXENT_NO_FP8=1")
    return d


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = [str(p) for p in ce.include_paths()]
    libdir = str(Path(torch.__file__).parent / "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def ext_path() -> Path:
    return PKG / f"_C{ext_suffix()}"


def _headers():
    return list((CSRC / "include").rglob("*.h")) + list((CSRC / "kernels").glob("*.h"))


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[-1] if cmd else cmd}")
    return r


def build(force: bool = False, cpp_targets: bool = True, verbose: bool = False) -> Path:
    BUILD.mkdir(exist_ok=True)
    (BUILD / "bin").mkdir(exist_ok=True)
    tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    common = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", f"-I{CSRC / 'include'}"]
    hdrs = _headers()

    k_objs = []
    t_src = CSRC / "runtime" / "ntxent_torch.cpp"
    t_obj = BUILD / "ntxent_torch.o"
    jobs = []
    for k_src in KERNEL_SRCS:
        k_obj = BUILD / (k_src.stem + ".o")
        k_objs.append(k_obj)
        if force or _stale(k_obj, [k_src, *hdrs]):
            jobs.append(common + ["-O3", "-c", str(k_src), "-o", str(k_obj)])
    if force or _stale(t_obj, [t_src, *hdrs]):
        tflags = [f"-I{p}" for p in tinc] + [
            f"-I{pyinc}",
            "-O2",
            "-DTORCH_EXTENSION_NAME=_C",
            "-DTORCH_API_INCLUDE_EXTENSION_H",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-DUSE_ROCM=1",
            "-Wno-unused-result",
            "-Wno-deprecated-declarations",
        ]
        # host-only translation unit: compile as plain C++ (no device pass over libtorch headers)
        hostc = _host_cxx() + [f"-I{CSRC / 'include'}"]
        jobs.append(hostc + tflags + ["-c", str(t_src), "-o", str(t_obj)])
    # native runtime (engine, RCCL communicator, tracing): host-only C++ against the HIP runtime
    rt_objs = []
    for name in RUNTIME_SRCS:
        src = CSRC / "runtime" / name
        obj = BUILD / (Path(name).stem + ".o")
        rt_objs.append(obj)
        if force or _stale(obj, [src, *hdrs]):
            jobs.append(_host_cxx() + [f"-I{CSRC / 'include'}", "-O2", *_feature_defines(), "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=4) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))

    so = ext_path()
    if force or _stale(so, [*k_objs, t_obj, *rt_objs]):
        # RCCL: bind to the copy torch ships (one RCCL instance per process)
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, k_objs), str(t_obj), *map(str, rt_objs),
                "-o", str(so), f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-ltorch_python", "-lrccl", "-ldl", f"-Wl,-rpath,{tlib}"]
        _run(link, verbose)

    if cpp_targets:
        build_cpp_targets([*k_objs, *rt_objs], force=force, verbose=verbose)
    return so


def cpp_test_sources():
    """Every source the C++ test executable is built from (its own file, the kernels, headers and
    the native runtime; not the torch binding)."""
    srcs = [ROOT / "tests" / "cpp" / "ntxent_tests.cpp", *KERNEL_SRCS, *_headers()]
    srcs += [CSRC / "runtime" / n for n in RUNTIME_SRCS]
    return sorted(srcs, key=lambda p: str(p.relative_to(ROOT)))


def source_hash(paths) -> str:
    """sha256 over (relative path, content) of ``paths``: what a binary was built from, independent
    of file mtimes (a fresh checkout resets them)."""
    import hashlib

    h = hashlib.sha256()
    for p in paths:
        h.update(str(p.relative_to(ROOT)).encode() + b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()


TESTS_HASH = BUILD / "bin" / "ntxent_tests.srchash"


def build_cpp_targets(objs, force: bool = False, verbose: bool = False):
    """Standalone C++ executables (no libtorch): benchmark + tests over the raw API."""
    hdrs = _headers()
    targets = {
        "ntxent_bench": ROOT / "bench" / "ntxent_bench.cpp",
        "ntxent_tests": ROOT / "tests" / "cpp" / "ntxent_tests.cpp",
    }
    def one(name, src):
        out = BUILD / "bin" / name
        obj = BUILD / f"{name}.o"
        if force or _stale(out, [src, *objs, *hdrs]):
            _run(_host_cxx() + [f"-I{CSRC / 'include'}", "-O2", *_feature_defines(), "-c", str(src), "-o", str(obj)],
                 verbose)
            _run([HIPCC, f"--offload-arch={ARCH}", str(obj), *map(str, objs), "-o", str(out), "-L/opt/rocm/lib",
                  "-lrccl", "-ldl", "-Wl,-rpath,/opt/rocm/lib"], verbose)

    with cf.ThreadPoolExecutor(max_workers=2) as ex:
        list(ex.map(lambda kv: one(*kv), [(n, s) for n, s in targets.items() if s.exists()]))
    # the sources the (now up-to-date) test binary was built from: tests/test_gpu_cpp_suite.py
    # refuses a binary whose recorded hash differs from the tree's
    TESTS_HASH.write_text(source_hash(cpp_test_sources()) + "\n")


SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-omit-frame-pointer", "-g"]


def build_sanitized(verbose: bool = False) -> Path:
    """Host-only ASan + UBSan build of the C++ tests: build/asan/ntxent_tests. Device code is
    not instrumented (GPU ASan is not available on the pool); the host runtime, plan building,
    arena carving and RCCL bootstrap are."""
    out_dir = BUILD / "asan"
    out_dir.mkdir(parents=True, exist_ok=True)
    inc = f"-I{CSRC / 'include'}"
    objs = []
    for k_src in KERNEL_SRCS:
        k_obj = out_dir / (k_src.stem + ".o")
        _run([HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", inc, "-O2", *SAN, "-c", str(k_src), "-o",
              str(k_obj)], verbose)
        objs.append(k_obj)
    for name in RUNTIME_SRCS:
        obj = out_dir / (Path(name).stem + ".o")
        _run(_host_cxx() + [inc, "-O1", *SAN, "-c", str(CSRC / "runtime" / name), "-o", str(obj)], verbose)
        objs.append(obj)
    t_obj = out_dir / "ntxent_tests.o"
    _run(_host_cxx() + [inc, "-O1", *SAN, "-c", str(ROOT / "tests" / "cpp" / "ntxent_tests.cpp"), "-o", str(t_obj)],
         verbose)
    exe = out_dir / "ntxent_tests"
    _run([HIPCC, f"--offload-arch={ARCH}", str(t_obj), *map(str, objs), "-o", str(exe), "-fsanitize=address",
          "-fsanitize=undefined", "-L/opt/rocm/lib", "-lrccl", "-ldl", "-Wl,-rpath,/opt/rocm/lib"], verbose)
    return exe


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--no-cpp", action="store_true")
    ap.add_argument("--asan", action="store_true", help="also build build/asan/ntxent_tests (host ASan+UBSan)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    so = build(force=a.force, cpp_targets=not a.no_cpp, verbose=a.verbose)
    print(f"built {so.relative_to(ROOT)}")
    if a.asan:
        print(f"built {build_sanitized(a.verbose).relative_to(ROOT)}")


if __name__ == "__main__":
    main()
