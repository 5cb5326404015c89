"""CPU tests of the product boundary: the C-ABI library loads and exports every declared symbol,
and the host-side PKO sampling tables reproduce libstdc++'s std::shuffle(mt19937(42)) prefix.
No GPU compute call happens here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import oracle
from lidar_odometry_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = "".join(open(os.path.join(ROOT, "include", h)).read() for h in sorted(os.listdir(os.path.join(ROOT, "include")))
                  if h.endswith(".h"))
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lo_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert sorted(_lib.EXPORTED_SYMBOLS) == _declared_symbols()


def test_library_exports_every_declared_symbol():
    L = C.CDLL(_lib.LIB_PATH)
    for name in _declared_symbols():
        assert hasattr(L, name), name


def test_library_is_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("n", [1, 2, 3, 7, 50, 99, 100, 101, 102, 255, 1000, 4096, 12345, 65534, 65535, 65536,
                               65537, 70001, 131072])
def test_pko_sample_indices_match_std_shuffle(n):
    L = _lib.lib()
    out = np.zeros(100, np.int32)
    k = L.lo_pko_sample_indices_host(n, 100, out.ctypes.data_as(C.POINTER(C.c_int32)))
    assert k == min(n, 100)
    np.testing.assert_array_equal(out[:k], oracle.shuffle_prefix(n, 100))


def test_pko_sample_indices_other_sample_sizes():
    L = _lib.lib()
    for S in (1, 17, 256):
        for n in (5, 300, 66000):
            out = np.zeros(S, np.int32)
            k = L.lo_pko_sample_indices_host(n, S, out.ctypes.data_as(C.POINTER(C.c_int32)))
            np.testing.assert_array_equal(out[:k], oracle.shuffle_prefix(n, S))


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    cfg = _lib.LoConfig()
    _lib.lib().lo_config_default_kitti(C.byref(cfg))
    err = C.c_int(0)
    ctx = _lib.lib().lo_create(C.byref(cfg), 0, C.byref(err))
    assert not ctx and err.value < 0
