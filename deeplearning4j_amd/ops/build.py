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
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(s, o, headers):
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
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", KERNEL_LIB] + objs)
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
