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
