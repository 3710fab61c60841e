"""CPU: the C-ABI library loads, exports every symbol include/super_rag_mi355x.h declares and no
diagnostic symbol (those are libsrmi_diag.so's, include/super_rag_mi355x_diag.h), and fails loudly
(no silent CPU fallback) when no GPU is visible."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header="super_rag_mi355x.h"):
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", header)).read(), flags=re.S)
    return set(re.findall(r"\b(sr_[a-z0-9_]+)\s*\(", src))


def _exports(path):
    import shutil
    import subprocess
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("sr_")}


def test_library_exports_every_declared_symbol():
    from super_rag_amd import _native
    lib = _native.load()
    declared = _declared()
    assert len(declared) >= 30
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert declared == set(_native.SIGNATURES), declared ^ set(_native.SIGNATURES)
    assert lib.sr_version() >= 100


def test_product_library_exports_no_diagnostic_symbol():
    # the sr_diag_* entry points (single-kernel drivers, timing-only variants,
    # the copy yardstick) are built into libsrmi_diag.so only; the product library exports exactly
    # the product header's functions
    from super_rag_amd import _native
    prod = _exports(_native.library_path())
    assert not [n for n in prod if n.startswith("sr_diag")], prod
    assert prod == _declared(), prod ^ _declared()
    diag = _declared("super_rag_mi355x_diag.h")
    assert diag == set(_native.DIAG_SIGNATURES) and all(n.startswith("sr_diag_") for n in diag)
    assert _exports(_native.diag_library_path()) == prod | diag
    lib = _native.load_diag()
    assert all(hasattr(lib, n) for n in diag)


def test_no_gpu_fails_loudly():
    from super_rag_amd import _native
    if _native.device_count() > 0:
        pytest.skip("GPU visible: covered by the gpu suite")
    from super_rag_amd.store import NativeStore
    with pytest.raises(_native.NativeUnavailableError):
        NativeStore(64)
    from super_rag_amd.encoder import MODELS, Encoder
    with pytest.raises(_native.NativeUnavailableError):
        Encoder(MODELS["bge-small-en"])


def test_error_codes_and_messages_without_device():
    import ctypes
    from super_rag_amd import _native
    lib = _native.load()
    h = ctypes.c_void_p()
    rc = lib.sr_store_create(0, 0, 16, ctypes.byref(h))   # invalid dim: checked before any HIP call
    assert rc == _native.SR_ERR_INVALID
    assert b"dim" in lib.sr_last_error()
    assert lib.sr_store_count(None, None, None) == _native.SR_ERR_INVALID
    stats = _native.profile_read()
    assert isinstance(stats, dict)


def test_library_has_no_unresolved_internal_symbols():
    """Every sr:: symbol the library references is defined in it: a launcher left inside an
    anonymous namespace links into the .so as an undefined symbol (lazy binding then fails only
    when the path is first called, on the GPU box)."""
    import shutil
    import subprocess
    from super_rag_amd import _native
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    out = subprocess.run([nm, "-D", "--undefined-only", _native.library_path()], capture_output=True,
                         text=True, check=True).stdout
    bad = [l.split()[-1] for l in out.splitlines() if "_ZN2sr" in l]
    assert not bad, bad
