"""The C-ABI library loads on a machine without a GPU and exports every symbol
declared in include/npge_amd.h (no compute calls here)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "npge_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(npgx_\w+)\s*\(", text)))


def test_library_exports_header_symbols():
    from npge_amd import build, _capi
    build.build()
    lib = ctypes.CDLL(_capi.LIB_PATH)
    names = _declared()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_no_device_fails_loudly_or_counts():
    from npge_amd import _capi
    L = _capi.lib()
    n = ctypes.c_int32(-1)
    assert L.npgx_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    if n.value == 0:
        h = ctypes.c_void_p()
        o = _capi.AfOptions()
        L.npgx_af_default_options(ctypes.byref(o))
        assert L.npgx_af_create(ctypes.byref(o), ctypes.byref(h)) == -3  # NPGX_ERR_NODEV
        assert b"no HIP device" in L.npgx_last_error()


def test_default_options_match_reference():
    from npge_amd import _capi
    L = _capi.lib()
    o = _capi.AfOptions()
    L.npgx_af_default_options(ctypes.byref(o))
    # CMakeLists.txt:41-45
    assert (o.anchor_size, o.anchor_fp_x1e4, o.anchor_similar, o.max_anchor_fragments) == \
        (20, 1000, 1, 100000)
    a = _capi.AlignOptions()
    L.npgx_align_default_options(ctypes.byref(a))
    # CMakeLists.txt:35-37,55-60
    assert (a.mismatch_check, a.gap_check, a.aligned_check, a.min_length, a.min_identity_x1e4) == \
        (1, 2, 10, 100, 9000)
