"""The drop-in boundary: libmvs.so loads on a CPU-only host and exports every
entry point include/mvs.h declares (no compute calls without a GPU)."""
import ctypes as C
import os
import re

import pytest

from cl_multiview_stereo_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "mvs.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mvs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_the_binding_lists():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_symbol():
    L = _lib.load()
    for name in declared():
        assert hasattr(L, name), name


def test_version_and_error_strings():
    L = _lib.load()
    assert b"gfx950" in L.mvs_version()
    assert isinstance(L.mvs_last_error(), bytes)


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = _lib.load()
    ctx = C.c_void_p()
    rc = L.mvs_create(0, C.byref(ctx))
    assert rc != 0 and not ctx.value
    assert len(L.mvs_last_error()) > 0


def test_null_context_is_rejected():
    L = _lib.load()
    assert L.mvs_synchronize(None) == -1
    assert L.mvs_cvt_d(None, None, 1, 4, 4, None, None) == -1


def test_engine_refuses_cpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cl_multiview_stereo_amd.engine import Engine
    with pytest.raises(_lib.MvsError):
        Engine(0)
