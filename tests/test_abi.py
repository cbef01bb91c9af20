"""C-ABI checks that need no GPU: the library loads and exports every symbol
include/tbdk.h declares (no compute calls)."""
import ctypes
import os
import re

from opencv_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "tbdk.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tbdk_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ["tbdk_ctx_create", "tbdk_pyr_build", "tbdk_lk_sparse", "tbdk_pyr_down_u8"]:
        assert must in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_covers_every_declared_symbol():
    assert set(declared_symbols()) == set(_lib.SIGNATURES), set(declared_symbols()) ^ set(_lib.SIGNATURES)


def test_version_and_no_device_error_path():
    lib = _lib.load()
    assert lib.tbdk_version().startswith(b"tbdk")
    # without a GPU, context creation must fail loudly with ENODEV (not fall back)
    import torch

    if not torch.cuda.is_available():
        h = ctypes.c_void_p()
        assert lib.tbdk_ctx_create(0, ctypes.byref(h)) == _lib.TBDK_ENODEV


def test_null_argument_validation_without_device():
    lib = _lib.load()
    assert lib.tbdk_ctx_destroy(None) == _lib.TBDK_EINVAL
    assert lib.tbdk_lk_sparse(None, None, None, None, None, None, None, None, 0, None, None) == _lib.TBDK_EINVAL
