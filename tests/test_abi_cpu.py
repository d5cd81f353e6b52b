"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/lnw.h declares; host-side constants match NumPy (no GPU needed)."""
import ctypes
import os
import re

import numpy as np
import pytest

import lnw
from lnw import _abi
from lnw.build import OUT, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    build()
    return _abi.load()


def header_symbols():
    src = open(os.path.join(ROOT, "include", "lnw.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|const char \*)\s*(lnw_\w+)\(", src, re.M)))


def test_header_symbols_match_binding():
    assert sorted(header_symbols()) == sorted(_abi.SYMBOLS)


def test_library_exports_every_header_symbol(L):
    for s in header_symbols():
        assert hasattr(L, s), s
    assert L.lnw_abi_version() == 5


def test_hit_tables_match_numpy(L):
    t64 = np.zeros(18)
    t32 = np.zeros(18, np.float32)
    assert L.lnw_hit_tables(t64.ctypes.data_as(ctypes.c_void_p),
                            t32.ctypes.data_as(ctypes.c_void_p)) == 0
    for h, p in enumerate((0.45, 0.63)):
        for n in range(9):
            # combatant.py:676-678 in float64 (np.float64 salvo) and float32 (np.float32 salvo)
            assert t64[h * 9 + n] == 1 - (1 - p) ** np.float64(n)
            assert t32[h * 9 + n] == np.float32(1 - (1 - p) ** np.float32(n))


def test_errors_are_reported_not_raised(L):
    p = _abi.Params()
    h = ctypes.c_void_p()
    rc = L.lnw_create(ctypes.byref(p), 16, 0, 2, 0, 0, ctypes.byref(h))
    assert rc == -5  # LNW_EUNSUPPORTED: nb must be >= 1
    assert b"ships per side" in L.lnw_last_error()
    assert L.lnw_step(None, None, 0, None, None, None, None, None, None, None, None) == -1


def test_product_path_has_no_cpu_fallback(tmp_path):
    """Loading from a missing path must raise, never fall back."""
    with pytest.raises(lnw.LnwError):
        _abi._lib = None
        _abi.load(str(tmp_path / "missing.so"))
    _abi._lib = None


def test_policy_entry_points_validate_arguments(L):
    """lnw_policy_act / lnw_rollout_post reject malformed arguments before
    touching the device (no GPU needed)."""
    assert L.lnw_policy_act(None, None) == -1
    assert L.lnw_rollout_post(None, None) == -1
    pa = _abi.PolicyArgs()  # no obs / params / alive
    assert L.lnw_policy_act(ctypes.byref(pa), None) == -1
    pp = _abi.RolloutPostArgs()
    pp.n = 0
    assert L.lnw_rollout_post(ctypes.byref(pp), None) == -1
