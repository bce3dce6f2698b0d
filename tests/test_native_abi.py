"""The C-ABI library loads and exports every symbol include/voxemb.h declares
(no GPU needed), and the host-only entry points behave."""

import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "voxemb.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vox_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_header():
    from voxsrc2020_speaker_verification_amd import _native
    lib = _native.lib()
    declared = _declared()
    assert len(declared) >= 19
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes table covers the header exactly
    assert sorted(_native.EXPORTED) == declared


def test_errors_are_reported():
    import ctypes as C
    from voxsrc2020_speaker_verification_amd import _native
    lib = _native.lib()
    h = C.c_void_p()
    rc = lib.vox_load(b"/nonexistent/blob", 0, 1, C.byref(h))
    assert rc == _native.VOX_EIO
    assert b"cannot open" in lib.vox_last_error()
    rc = lib.vox_load_blob(b"garbage!" * 4, 32, 0, 1, C.byref(h))
    assert rc == _native.VOX_EIO
    with pytest.raises(_native.VoxError):
        _native.check(rc)


def test_bad_blob_rejected_before_device():
    """A malformed blob fails at parse time (no GPU is touched)."""
    import ctypes as C
    from voxsrc2020_speaker_verification_amd import _native
    blob = b"VOXEMB01" + (10 ** 9).to_bytes(8, "little")
    h = C.c_void_p()
    assert _native.lib().vox_load_blob(blob, len(blob), 0, 1, C.byref(h)) == _native.VOX_EIO


def test_kernel_param_mirrors_match_the_library():
    """The GPU unit tests launch bneck_fused / gconv3x3_rows through ctypes
    mirrors of their parameter structs: a mirror shorter than the C++ struct
    makes the kernel read past it (round 6: an illegal address when
    BneckParams grew).  Their sizes must equal the library's."""
    import ctypes as C
    import importlib.util
    import os
    from voxsrc2020_speaker_verification_amd._native import lib
    here = os.path.dirname(os.path.abspath(__file__))
    for which, (mod, cls) in enumerate([("test_bneck_unit", "BneckParams"),
                                         ("test_gconv_unit", "GconvParams")]):
        spec = importlib.util.spec_from_file_location(mod, os.path.join(here, mod + ".py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        assert C.sizeof(getattr(m, cls)) == lib().vox_debug_struct_size(which), cls
