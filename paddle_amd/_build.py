"""In-tree native build for paddle_amd.

Two native artefacts, both built in place so they travel with the repo snapshot:

* ``paddle_amd/lib/libpaddle_amd_kernels.so`` -- the CDNA4 (gfx950) HIP kernel
  library (``csrc/kernels/*.hip``), compiled with ``hipcc --offload-arch=gfx950``.
  It exposes a flat C ABI (``pa_*`` launchers taking raw device pointers and a
  ``hipStream_t``) so it has no dependency on PyTorch headers and compiles in
  seconds.
* ``paddle_amd/lib/libpaddle_amd_runtime.so`` -- the C++17 runtime
  (``csrc/runtime/*.cc``): buddy allocator, LoDTensor stream serialisation,
  RecordIO, thread pool / blocking queue, SSA dependency scheduler, profiler
  event buffers.  Plain C ABI as well, bound with ctypes.

Object files are cached under ``build/`` keyed by source mtime + flags, and the
link step is skipped when the library is newer than every object.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
LIBDIR = os.path.join(ROOT, "lib")
BUILDDIR = os.path.join(REPO, "build", "native")
ARCH = os.environ.get("PADDLE_AMD_ARCH", "gfx950")

KERNEL_LIB = os.path.join(LIBDIR, "libpaddle_amd_kernels.so")
RUNTIME_LIB = os.path.join(LIBDIR, "libpaddle_amd_runtime.so")
NATIVE_LIB = os.path.join(LIBDIR, "libpaddle_amd_native.so")
NATIVE_INC = os.path.join(ROOT, "csrc", "native")
TRACER_LIB = os.path.join(LIBDIR, "libpaddle_amd_tracer.so")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the paddle_amd kernel library needs ROCm's hipcc")


def _torch_lib_dir() -> str | None:
    try:
        import torch  # noqa: F401

        return os.path.join(os.path.dirname(torch.__file__), "lib")
    except Exception:  # pragma: no cover
        return None


def _needs(obj: str, deps: list[str], stamp: str) -> bool:
    if not os.path.exists(obj) or not os.path.exists(obj + ".flags"):
        return True
    if open(obj + ".flags").read() != stamp:
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(cmd: list[str], obj: str, stamp: str, verbose: bool):
    if verbose:
        print("[paddle_amd build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed for {obj}:\n{r.stderr[-6000:]}")
    with open(obj + ".flags", "w") as f:
        f.write(stamp)


def _build_lib(srcs, hdrs, out, compiler, cflags, ldflags, verbose, jobs):
    os.makedirs(BUILDDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    objs, todo = [], []
    stamp = hashlib.sha1(" ".join([compiler] + cflags).encode()).hexdigest()
    for s in srcs:
        obj = os.path.join(BUILDDIR, os.path.basename(s) + ".o")
        objs.append(obj)
        if _needs(obj, [s] + hdrs, stamp):
            todo.append(([compiler] + cflags + ["-c", s, "-o", obj], obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(lambda a: _compile(a[0], a[1], stamp, verbose), todo))
    if todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [compiler, "-shared", "-o", out + ".tmp"] + objs + ldflags
        if verbose:
            print("[paddle_amd build]", " ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed for {out}:\n{r.stderr[-4000:]}")
        os.replace(out + ".tmp", out)
    return out


def build_kernels(verbose: bool = False, jobs: int | None = None) -> str:
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h")))
    cflags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-fvisibility=hidden",
              "-ffp-contract=fast", "-munsafe-fp-atomics"]
    ldflags = [f"--offload-arch={ARCH}"]
    tl = _torch_lib_dir()
    if tl:
        # link the same libamdhip64 (SONAME libamdhip64.so.7) torch itself loads
        ldflags += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
    ldflags += ["-lamdhip64"]
    return _build_lib(srcs, hdrs, KERNEL_LIB, _hipcc(), cflags, ldflags, verbose,
                      jobs or min(8, os.cpu_count() or 4))


def build_runtime(verbose: bool = False, jobs: int | None = None) -> str:
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.cc")))
    if not srcs:
        return ""
    hdrs = sorted(glob.glob(os.path.join(ROOT, "csrc", "runtime", "*.h")))
    cxx = shutil.which("g++") or "c++"
    cflags = ["-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall", "-pthread",
              "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    ldflags = ["-pthread", "-lz", "-ldl"]
    tl = _torch_lib_dir()
    if tl:
        ldflags += [f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64"]
    else:
        ldflags += ["-L/opt/rocm/lib", "-lamdhip64"]
    extra = os.environ.get("PADDLE_AMD_RUNTIME_CFLAGS", "").split()
    return _build_lib(srcs, hdrs, RUNTIME_LIB, cxx, cflags + extra, ldflags, verbose,
                      jobs or min(8, os.cpu_count() or 4))


def _hip_ldflags() -> list[str]:
    tl = _torch_lib_dir()
    if tl:  # the same libamdhip64 torch loads, so ctypes users share one HIP runtime
        return [f"-L{tl}", f"-Wl,-rpath,{tl}", "-lamdhip64"]
    return ["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lamdhip64"]


def build_native(verbose: bool = False, jobs: int | None = None) -> str:
    """The native C++ executor + inference API (``csrc/native``): host kernels
    compiled with g++ (AVX2/FMA), device glue kernels with hipcc for gfx950, one
    shared library with public C++ symbols (paddle_inference_api.h) and a C ABI,
    linked against the kernel library for GEMM / conv / pool / norm / loss /
    optimizer kernels."""
    d = os.path.join(ROOT, "csrc", "native")
    ccs = sorted(glob.glob(os.path.join(d, "*.cc")))
    hips = sorted(glob.glob(os.path.join(d, "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(d, "*.h")))
    os.makedirs(BUILDDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    cxx = shutil.which("g++") or "c++"
    ccflags = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-pthread", "-mavx2", "-mfma",
               "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    hipflags = ["-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-ffp-contract=fast"]
    objs, todo = [], []
    for srcs, comp, fl in ((ccs, cxx, ccflags), (hips, _hipcc(), hipflags)):
        stamp = hashlib.sha1(" ".join([comp] + fl).encode()).hexdigest()
        for s in srcs:
            obj = os.path.join(BUILDDIR, "native_" + os.path.basename(s) + ".o")
            objs.append(obj)
            if _needs(obj, [s] + hdrs, stamp):
                todo.append(([comp] + fl + ["-c", s, "-o", obj], obj, stamp))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
            list(ex.map(lambda a: _compile(a[0], a[1], a[2], verbose), todo))
    out = NATIVE_LIB
    # the device kernels call the shared kernel library (csrc/native/kernel_lib.h):
    # link it, found next to this library at run time ($ORIGIN)
    klib = build_kernels(verbose, jobs)
    if (todo or not os.path.exists(out) or os.path.getmtime(klib) > os.path.getmtime(out)
            or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs)):
        cmd = ([_hipcc(), "-shared", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs + ["-pthread"]
               + [f"-L{LIBDIR}", "-lpaddle_amd_kernels", "-Wl,-rpath,$ORIGIN"] + _hip_ldflags())
        if verbose:
            print("[paddle_amd build]", " ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed for {out}:\n{r.stderr[-4000:]}")
        os.replace(out + ".tmp", out)
    return out


FASTOPS_LIB = os.path.join(LIBDIR, "pa_fastops.so")


def build_fastops(verbose: bool = False) -> str:
    """The C++ launch entry for the hot elementwise ops (``csrc/fastops``): a CPython
    extension against torch's C++ API (tensor unpacking without Python) that calls
    the kernel library's ``pa_ew_flat``.  Optional: skipped when torch's headers are
    not available."""
    src = os.path.join(ROOT, "csrc", "fastops", "fastops.cc")
    if not os.path.exists(src):
        return ""
    import sysconfig

    import torch
    from torch.utils import cpp_extension as ce

    klib = build_kernels(verbose)
    out = FASTOPS_LIB
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = ["-O2", "-fPIC", "-std=c++17", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-DTORCH_EXTENSION_NAME=pa_fastops", "-DTORCH_API_INCLUDE_EXTENSION_H", "-w"]
    flags += [f"-I{p}" for p in ce.include_paths()] + [f"-I{sysconfig.get_paths()['include']}"]
    flags += ["-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]  # the HIP runtime headers c10/hip/HIPStream.h needs
    tl = _torch_lib_dir()
    libs = [f"-L{tl}", f"-Wl,-rpath,{tl}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            f"-L{LIBDIR}", "-lpaddle_amd_kernels", "-Wl,-rpath,$ORIGIN"]
    stamp = hashlib.sha1(" ".join(flags + libs).encode()).hexdigest()
    if not _needs(out, [src, klib], stamp):
        return out
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx] + flags + [src, "-o", out + ".tmp"] + libs
    if verbose:
        print("[paddle_amd build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"fastops build failed:\n{r.stderr[-4000:]}")
    os.replace(out + ".tmp", out)
    with open(out + ".flags", "w") as f:
        f.write(stamp)
    return out


def build_native_program(src: str, out: str, extra: list[str] | None = None) -> str:
    """Compiles a C++ program against the native library's public headers
    (paddle_inference_api.h / framework.h) and links libpaddle_amd_native.so."""
    lib = build_native()
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-O2", "-std=c++17", "-pthread", src, f"-I{NATIVE_INC}", f"-L{LIBDIR}", "-lpaddle_amd_native",
           f"-Wl,-rpath,{LIBDIR}", "-o", out] + (extra or [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"building {src} failed:\n{r.stderr[-4000:]}")
    assert os.path.exists(lib)
    return out


def build_tracer(verbose: bool = False) -> str:
    """The in-process kernel activity tracer (``csrc/tracer``): a rocprofiler-sdk
    tool library (host C++ only, linked against librocprofiler-sdk)."""
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "tracer", "*.cc")))
    if not srcs or not os.path.exists("/opt/rocm/include/rocprofiler-sdk/rocprofiler.h"):
        return ""
    cxx = shutil.which("g++") or "c++"
    cflags = ["-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall", "-pthread",
              "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    ldflags = ["-pthread", "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-lrocprofiler-sdk"]
    return _build_lib(srcs, [], TRACER_LIB, cxx, cflags, ldflags, verbose, 1)


def core_ext_path() -> str:
    import sysconfig

    return os.path.join(LIBDIR, "paddle_amd_core" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


def build_core_ext(verbose: bool = False) -> str:
    """The CPython extension ``paddle_amd_core`` (csrc/pybind): pybind11 bindings of
    the native C++ ProgramDesc / Scope / LoDTensor / Executor (the reference's
    pybind core), linked against libpaddle_amd_native.so."""
    try:
        import sysconfig

        import pybind11
    except ImportError:
        return ""
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "pybind", "*.cc")))
    if not srcs:
        return ""
    native_lib = build_native(verbose)
    out = core_ext_path()
    hdrs = sorted(glob.glob(os.path.join(ROOT, "csrc", "native", "*.h")))
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(f) for f in srcs + hdrs + [native_lib]):
        return out
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", f"-I{pybind11.get_include()}",
           f"-I{sysconfig.get_paths()['include']}", "-I/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"] + srcs + \
        ["-o", out + ".tmp", f"-L{LIBDIR}", "-lpaddle_amd_native", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print("[paddle_amd build]", " ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"building {out} failed:\n{r.stderr[-4000:]}")
    os.replace(out + ".tmp", out)
    return out


def build_all(verbose: bool = False) -> list[str]:
    out = [build_kernels(verbose)]
    rt = build_runtime(verbose)
    if rt:
        out.append(rt)
    out.append(build_native(verbose))
    tr = build_tracer(verbose)
    if tr:
        out.append(tr)
    ce = build_core_ext(verbose)
    if ce:
        out.append(ce)
    fo = build_fastops(verbose)
    if fo:
        out.append(fo)
    return out


if __name__ == "__main__":
    for p in build_all(verbose="-v" in sys.argv):
        print(p)
