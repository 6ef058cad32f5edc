"""CPU: the C-ABI library loads and exports every function include/fdengine.h declares; host-only
entry points behave (no compute calls that need a GPU)."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
HEADER = REPO / "include" / "fdengine.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(fd_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_core_api():
    names = declared_functions()
    for core in ("fd_engine_create", "fd_load_forest", "fd_forest_predict_device", "fd_blend_device",
                 "fd_last_error", "fd_pack_forest_host"):
        assert core in names


def test_library_exports_every_declared_symbol():
    from fdengine import _native as N
    lib = C.CDLL(str(N.LIB_PATH))
    missing = [f for f in declared_functions() if not hasattr(lib, f)]
    assert not missing, missing
    # and the Python binding covers the whole header
    assert set(declared_functions()) <= set(N.SIGNATURES), set(declared_functions()) - set(N.SIGNATURES)


def test_abi_version_and_error_path():
    from fdengine import _native as N
    assert N.lib.fd_abi_version() == 15
    # null engine -> status code + message, no exception across the ABI
    rc = N.lib.fd_engine_sync(None)
    assert rc == N.FD_ERR_INVALID_ARG
    assert b"null engine" in N.lib.fd_last_error()


def test_pack_rejects_bad_trees():
    from fdengine import ForestArrays, _native as N
    from fdengine.engine import pack_forest_host
    good = dict(kind=N.FD_FOREST_XGB_BINARY_LOGISTIC, num_feature=4, offsets=np.array([0, 3]),
                left=np.array([1, -1, -1]), right=np.array([2, -1, -1]), feature=np.array([0, 0, 0]),
                threshold=np.array([0.5, 0, 0]), default_left=np.array([1, 0, 0]),
                leaf_value=np.array([0, 1.0, -1.0]))
    blob, ids, info = pack_forest_host(ForestArrays(**good))
    assert info.depth == 1 and info.n_trees == 1
    bad = dict(good, feature=np.array([9, 0, 0]))  # split feature >= num_feature
    with pytest.raises(N.NativeError):
        pack_forest_host(ForestArrays(**bad))
    cyc = dict(good, left=np.array([0, -1, -1]))  # cycle
    with pytest.raises(N.NativeError):
        pack_forest_host(ForestArrays(**cyc))
    deep_n = 25  # a chain deeper than the supported maximum (10)
    left = np.array([i + 1 if i < deep_n - 1 else -1 for i in range(deep_n)] + [-1] * (deep_n - 1))
    right = np.array([deep_n + i if i < deep_n - 1 else -1 for i in range(deep_n)] + [-1] * (deep_n - 1))
    m = len(left)
    deep = dict(good, offsets=np.array([0, m]), left=left, right=right, feature=np.zeros(m, int),
                threshold=np.zeros(m), default_left=np.zeros(m, int), leaf_value=np.zeros(m))
    with pytest.raises(N.NativeError) as ei:
        pack_forest_host(ForestArrays(**deep))
    assert ei.value.code == N.FD_ERR_UNSUPPORTED
