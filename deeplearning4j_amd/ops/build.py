"""Build the native libraries in-tree (no JIT cache, so the .so travels with the repo snapshot).

* ``libdl4j_amd_kernels.so`` — every ``csrc/*.hip`` compiled for gfx950 with hipcc (C ABI, ctypes).
* ``libdl4j_amd_runtime.so`` — host-only C++ runtime pieces (``csrc/runtime/*.cpp``: threshold codec,
  data-loader helpers, trees/t-SNE helpers), compiled with g++.
Incremental: an object is rebuilt only when its source or any header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "deeplearning4j_amd", "_lib")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
KERNEL_LIB = os.path.join(LIBDIR, "libdl4j_amd_kernels.so")
RUNTIME_LIB = os.path.join(LIBDIR, "libdl4j_amd_runtime.so")


def _local_includes(src, seen=None):
    """Headers a source pulls in with #include "..." (recursively, resolved next to the including file): a
    source is rebuilt only when one of ITS headers changed."""
    import re
    seen = set() if seen is None else seen
    try:
        text = open(src).read()
    except OSError:
        return seen
    for name in re.findall(r'^\s*#\s*include\s+"([^"]+)"', text, re.M):
        h = os.path.normpath(os.path.join(os.path.dirname(src), name))
        if h not in seen and os.path.exists(h):
            seen.add(h)
            _local_includes(h, seen)
    return seen


def _newer(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(h) > t for h in headers)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_kernels(verbose=True, jobs=None):
    os.makedirs(LIBDIR, exist_ok=True)
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(s, o, sorted(_local_includes(s))):
            todo.append((s, o))
    flags = ["-O3", "-fPIC", f"--offload-arch={ARCH}", "-std=c++17", "-munsafe-fp-atomics", "-I", CSRC]
    jobs = jobs or min(8, os.cpu_count() or 4, 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = {ex.submit(_run, [HIPCC] + flags + ["-c", s, "-o", o]): s for s, o in todo}
        for f in cf.as_completed(futs):
            f.result()
            if verbose:
                print(f"[build] compiled {os.path.basename(futs[f])}", file=sys.stderr)
    if todo or not os.path.exists(KERNEL_LIB):
        # librccl: the C ABI's communicator entry points (csrc/abi.hip dl4j_comm_*)
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", KERNEL_LIB] + objs +
             ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
        if verbose:
            print(f"[build] linked {KERNEL_LIB}", file=sys.stderr)
    return KERNEL_LIB


def build_runtime(verbose=True):
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return None
    os.makedirs(LIBDIR, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if os.path.exists(RUNTIME_LIB) and not any(_newer(s, RUNTIME_LIB, headers) for s in srcs):
        return RUNTIME_LIB
    _run(["g++", "-O3", "-fPIC", "-shared", "-std=c++17", "-pthread", "-o", RUNTIME_LIB] + srcs)
    if verbose:
        print(f"[build] linked {RUNTIME_LIB}", file=sys.stderr)
    return RUNTIME_LIB


ABI_DRIVER = os.path.join(ROOT, "tests", "native", "abi_driver")


def build_abi_driver(verbose=True):
    """The C-only driver of the public ABI (tests/native/abi_driver.c against csrc/include/dl4j_amd.h): plain gcc,
    C99, linked with both in-tree libraries (rpath to them) and libamdhip64."""
    src = ABI_DRIVER + ".c"
    hdr = os.path.join(CSRC, "include", "dl4j_amd.h")
    if not os.path.exists(src):
        return None
    deps = [src, hdr, KERNEL_LIB, RUNTIME_LIB]
    if os.path.exists(ABI_DRIVER) and all(os.path.getmtime(d) <= os.path.getmtime(ABI_DRIVER) for d in deps
                                          if os.path.exists(d)):
        return ABI_DRIVER
    _run(["gcc", "-std=c99", "-O2", "-Wall", "-I", os.path.join(CSRC, "include"), src, "-o", ABI_DRIVER,
          "-L", LIBDIR, "-ldl4j_amd_kernels", "-ldl4j_amd_runtime", f"-Wl,-rpath,{LIBDIR}", "-L/opt/rocm/lib",
          "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib", "-lm"])
    if verbose:
        print(f"[build] linked {ABI_DRIVER}", file=sys.stderr)
    return ABI_DRIVER


SANITIZERS = ("address", "thread", "undefined")


def build_runtime_sanitized(kind, verbose=True):
    """Standalone self-test executable of the host runtime built with ``-fsanitize=<kind>`` (address / thread /
    undefined): every csrc/runtime/*.cpp plus csrc/runtime/tests/selftest.cpp. A sanitizer cannot instrument a
    ctypes-loaded library inside an uninstrumented Python, so the runtime is exercised by its own driver."""
    if kind not in SANITIZERS:
        raise ValueError(f"sanitize must be one of {SANITIZERS}")
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    drv = os.path.join(CSRC, "runtime", "tests", "selftest.cpp")
    out_dir = os.path.join(BUILD, f"san_{kind}")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "runtime_selftest")
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if os.path.exists(exe) and not any(_newer(s, exe, headers) for s in srcs + [drv]):
        return exe
    flags = ["-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={kind}", "-std=c++17", "-pthread"]
    if kind == "undefined":
        flags.append("-fno-sanitize-recover=all")
    _run(["g++"] + flags + ["-o", exe] + srcs + [drv])
    if verbose:
        print(f"[build] {exe}", file=sys.stderr)
    return exe


def build_all(verbose=True):
    k = build_kernels(verbose)
    r = build_runtime(verbose)
    build_abi_driver(verbose)
    return k, r


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--sanitize", choices=SANITIZERS, default=None,
                    help="build the host-runtime self-test under a sanitizer instead of the libraries")
    a = ap.parse_args()
    if a.sanitize:
        print(build_runtime_sanitized(a.sanitize))
    else:
        build_all()
