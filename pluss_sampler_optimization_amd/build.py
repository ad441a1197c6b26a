"""Build libpluss_gpu.so (gfx950) in-tree with hipcc.

The shared library is the product: the C ABI of include/pluss_gpu.h over the
HIP kernels in csrc/.  It is built next to this file (lib/) so it travels
with the repository snapshot to the GPU box.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libpluss_gpu.so")
HOST_LIB = os.path.join(LIBDIR, "libpluss_host.so")
HOST_SOURCES = ["host/pluss_host.cpp"]
CLI = os.path.join(LIBDIR, "pluss_cli")
ARCH = os.environ.get("PLUSS_OFFLOAD_ARCH", "gfx950")
SOURCES = ["pluss_kernels.hip", "pluss_faithful.hip", "pluss_fa_w32.hip", "pluss_fa_w64.hip", "pluss_fa_w32p.hip",
           "pluss_fa_smp.hip",
           "pluss_fa_gen.hip", "pluss_fa_uni.hip", "pluss_uniform.hip", "pluss_group.hip",
           "pluss_capi.hip"]
HEADERS = ["pluss_model.h", "pluss_internal.h", "pluss_device.h", "pluss_faithful.h", "pluss_sort.h", "pluss_uniform.h"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the PLUSS GPU library needs ROCm's hipcc")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose=False, force=False, variant=None):
    """variant "stages": the diagnostic build (-DPLUSS_DEBUG_STAGES: each named
    stage drains its stream and prints its outcome) into lib/stages/, for
    tools that load it explicitly; never the product library."""
    if variant == "stages":
        return _build_gpu(os.path.join(LIBDIR, "stages", "obj"), os.path.join(LIBDIR, "stages", "libpluss_gpu.so"),
                          ["-DPLUSS_DEBUG_STAGES"], verbose, force, SOURCES + ["diag/pluss_stages.hip"])
    lib = _build_gpu(OBJDIR, LIB, [], verbose, force, SOURCES)
    _build_host(verbose, force)
    return lib


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def _build_gpu(objdir, libpath, extra, verbose, force, sources):
    os.makedirs(objdir, exist_ok=True)
    hipcc = _hipcc()
    inc = os.path.join(HERE, "..", "include")
    common_deps = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(inc, "pluss_gpu.h"),
                                                              os.path.join(inc, "pluss_diag.h"), __file__]
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", inc, "-I", CSRC,
             "-Wall", "-Wno-unused-result", *extra]
    jobs = []
    objs = []
    for src in sources:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        objs.append(o)
        if force or _stale(o, [s] + common_deps):
            jobs.append([hipcc, *flags, "-c", s, "-o", o])

    with ThreadPoolExecutor(max_workers=len(jobs) or 1) as ex:
        list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _stale(libpath, objs):
        _run([hipcc, "-shared", f"--offload-arch={ARCH}", "-o", libpath, *objs], verbose)
    return libpath


def _build_host(verbose, force):
    inc = os.path.join(HERE, "..", "include")
    run = lambda c: _run(c, verbose)  # noqa: E731
    # host half of the pipeline (CRI / AET / formats): plain C++, no HIP
    hsrc = [os.path.join(CSRC, h) for h in HOST_SOURCES]
    if force or _stale(HOST_LIB, hsrc + [os.path.join(inc, "pluss_host.h"), os.path.join(inc, "pluss_gpu.h")]):
        run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-I", inc,
             "-o", HOST_LIB, *hsrc])
    # the reference's drivers (acc / speed / sample / replay) over both libraries
    csrc_cli = os.path.join(CSRC, "host", "pluss_cli.cpp")
    if force or _stale(CLI, [csrc_cli, LIB, HOST_LIB]):
        run([os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-Wall", "-I", inc, "-o", CLI, csrc_cli,
             "-L", LIBDIR, "-lpluss_gpu", "-lpluss_host", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"])


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv, variant="stages" if "--stages" in sys.argv else None))
