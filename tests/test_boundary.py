"""CPU checks of the drop-in boundary: the C-ABI libraries load and export
every symbol the headers declare, and the product library reads no
environment variable (no CPU fallback, no hidden knobs).  No compute call is
made here (no GPU in this container)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
CSRC = os.path.join(ROOT, "pluss_sampler_optimization_amd", "csrc")
LIB = os.path.join(ROOT, "pluss_sampler_optimization_amd", "lib", "libpluss_gpu.so")
HOST_LIB = os.path.join(ROOT, "pluss_sampler_optimization_amd", "lib", "libpluss_host.so")


def declared(header):
    txt = open(os.path.join(INC, header)).read()
    return sorted(set(re.findall(r"^(?:int|void|const char)\s*\**\s*(pluss_\w+)\s*\(", txt, re.M)))


@pytest.mark.parametrize("header,lib", [("pluss_gpu.h", LIB), ("pluss_diag.h", LIB), ("pluss_host.h", HOST_LIB)])
def test_library_exports_every_declared_symbol(header, lib):
    if not os.path.exists(lib):
        pytest.skip("library not built (python -m pluss_sampler_optimization_amd.build)")
    names = declared(header)
    assert names
    L = ctypes.CDLL(lib)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_python_binding_covers_the_headers():
    from pluss_sampler_optimization_amd import _lib
    assert sorted(_lib.EXPORTS) == declared("pluss_gpu.h")
    assert sorted(_lib.DIAG_EXPORTS) == declared("pluss_diag.h")


def test_product_reads_no_environment():
    """No getenv in the library's own sources, and no PLUSS_* variable name in
    the built library (rocPRIM's own ROCPRIM_* lookups are its business)."""
    for f in os.listdir(CSRC):
        if f.endswith((".hip", ".h", ".cpp")):
            assert "getenv" not in open(os.path.join(CSRC, f)).read(), f
    for f in os.listdir(os.path.join(CSRC, "host")):
        assert "getenv" not in open(os.path.join(CSRC, "host", f)).read(), f
    if os.path.exists(LIB):
        out = subprocess.run(["strings", LIB], capture_output=True, text=True).stdout
        assert "PLUSS_" not in out.replace("PLUSS_ERR", "").replace("PLUSS_OK", "")


# Kernels still allowed to request scratch (private segment), each with the
# reason; the list only shrinks.  No product kernel may request scratch: on
# gfx950 under ROCm 7's scratch reclaim, a kernel that does, running while the
# process's other HSA queues hold work, faulted the device (r5p, DESIGN.md
# section 8).
SCRATCH_ALLOWED = {}


def kernel_resources(lib):
    """{kernel symbol: private segment bytes} of the gfx950 code objects in a
    HIP shared library (llvm-readelf on the unbundled device image)."""
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    if not os.path.exists(os.path.join(llvm, "clang-offload-bundler")):
        pytest.skip("ROCm LLVM tools not installed")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        r = subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x")],
                           capture_output=True)
        assert r.returncode == 0, r.stderr
        blob = open(fat, "rb").read()
        # the fat binary holds one clang offload bundle per translation unit
        starts = [m.start() for m in re.finditer(rb"__CLANG_OFFLOAD_BUNDLE__", blob)]
        for k, a in enumerate(starts):
            part = os.path.join(d, f"b{k}.bin")
            open(part, "wb").write(blob[a:starts[k + 1] if k + 1 < len(starts) else len(blob)])
            co = os.path.join(d, f"k{k}.co")
            r = subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co):
                continue
            notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
            for b in notes.split(".agpr_count")[1:]:
                name = re.search(r"\.name:\s+(\S+)", b)
                priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", b)
                if name and priv:
                    out[name.group(1)] = int(priv.group(1))
    return out


def test_no_product_kernel_requests_scratch():
    if not os.path.exists(LIB):
        pytest.skip("library not built (python -m pluss_sampler_optimization_amd.build)")
    res = kernel_resources(LIB)
    assert len(res) > 50, len(res)  # (every translation unit's kernels were read)
    bad = {k: v for k, v in res.items() if v and not any(a in k for a in SCRATCH_ALLOWED)}
    assert not bad, bad
