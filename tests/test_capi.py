"""The C-ABI library loads and exports every symbol include/plba.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(plba_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from plba import lib
    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libplba.so not built (run __graft_entry__.build())")
    L = ctypes.CDLL(lib.LIB_PATH)
    names = _declared("plba.h")
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(lib.EXPORTED) <= set(names)


def test_create_fails_loudly_without_gpu():
    import torch  # noqa: F401  (only to probe for a device without initialising HIP ourselves)
    from plba import lib
    if not os.path.exists(lib.LIB_PATH):
        pytest.skip("libplba.so not built")
    if os.environ.get("HIP_VISIBLE_DEVICES", None) is None and os.path.exists("/dev/kfd"):
        pytest.skip("a GPU may be present; this test is for the CPU-only container")
    with pytest.raises(lib.PlbaError):
        lib.Solver()


def test_missing_library_raises(tmp_path):
    from plba import lib
    saved = lib._lib
    lib._lib = None
    try:
        with pytest.raises(lib.PlbaError):
            lib.load(str(tmp_path / "nope.so"))
    finally:
        lib._lib = saved
