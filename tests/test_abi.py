"""The C ABI boundary: libuwvk.so loads and exports every function that
include/uwvk.h declares; without a GPU every handle creation fails loudly
(no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

from uwvk import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "uwvk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(uwvk_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_symbols():
    assert sorted(engine.SYMBOLS) == header_functions()


def test_library_exports_every_symbol():
    if not os.path.exists(engine.LIB_PATH):
        pytest.skip("libuwvk.so not built (run __graft_entry__.build())")
    L = C.CDLL(engine.LIB_PATH)
    missing = [s for s in header_functions() if not hasattr(L, s)]
    assert not missing, missing
    assert L.uwvk_abi_version() == engine.ABI_VERSION == 3


def test_no_cpu_fallback():
    if not os.path.exists(engine.LIB_PATH):
        pytest.skip("libuwvk.so not built")
    if engine.device_available(0):
        pytest.skip("a GPU is present")
    with pytest.raises(engine.UWVKError) as e:
        engine.PoseUKFBatch(4)
    assert e.value.code == 5  # UWVK_EDEVICE
    with pytest.raises(engine.UWVKError):
        engine.VelocityUKFBatch(4)
