"""The C-ABI library loads without a GPU and exports every symbol include/*.h declares."""
import glob
import os
import re

from conftest import ROOT


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(slam_[a-z0-9_]+)\s*\(", src))
    return names


def test_header_declares_entry_points():
    d = _declared()
    assert {"slam_hamming_knn2", "slam_ba_iterate", "slam_last_error"} <= d


def test_library_exports_all_declared_symbols():
    from slam355 import _lib

    missing = [n for n in sorted(_declared()) if not hasattr(_lib.lib, n)]
    assert not missing, missing
    # every declared symbol has a ctypes signature (so no call goes through untyped)
    assert not (_declared() - set(_lib.SIGNATURES)), sorted(_declared() - set(_lib.SIGNATURES))
    assert _lib.lib.slam_abi_version() == 1


def test_no_gpu_error_paths():
    """Argument errors surface as status codes + messages without touching a GPU."""
    from slam355 import _lib

    rc = _lib.lib.slam_hamming_knn2(None, None, 10, None, None, 70000, 1, None, None, None, None)
    assert rc == -1 and b"t_cap" in _lib.lib.slam_last_error()
    rc = _lib.lib.slam_hamming_knn2(None, None, 10, None, None, 10, 1, None, None, None, None)
    assert rc == -1 and b"null" in _lib.lib.slam_last_error()
