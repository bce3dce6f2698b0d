"""ctypes binding of libvoxemb.so (include/voxemb.h).

There is no fallback: if the in-tree library is missing or fails to load, every
entry point raises `NativeUnavailable`.  Build it with
`python -m voxsrc2020_speaker_verification_amd.build_native` (or
`__graft_entry__.build()`).
"""

from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VOXEMB_LIB", os.path.join(HERE, "libvoxemb.so"))

VOX_OK = 0
VOX_EINVAL = -22
VOX_ENOMEM = -12
VOX_EIO = -5
VOX_ESHORT = -61
VOX_EHIP = -1000
VOX_FP32 = 0
VOX_BF16 = 1

# (name, restype, argtypes) -- must mirror include/voxemb.h
_P = C.c_void_p
_F = C.POINTER(C.c_float)


class FbankOpts(C.Structure):
    """vox_fbank_opts (include/voxemb.h)."""
    _fields_ = [("sample_frequency", C.c_float), ("frame_length_ms", C.c_float),
                ("frame_shift_ms", C.c_float), ("dither", C.c_float),
                ("preemphasis_coefficient", C.c_float), ("remove_dc_offset", C.c_int),
                ("num_mel_bins", C.c_int), ("low_freq", C.c_float), ("high_freq", C.c_float),
                ("seed", C.c_uint64)]


class Tap(C.Structure):
    """vox_tap (include/voxemb.h): one layer output of the plan."""
    _fields_ = [("op_end", C.c_int), ("n", C.c_int), ("h", C.c_int), ("w", C.c_int),
                ("c", C.c_int), ("ld", C.c_int), ("dtype", C.c_int), ("data", C.c_void_p)]


_FO = C.POINTER(FbankOpts)
_SIGS = [
    ("vox_load", C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(_P)]),
    ("vox_load_blob", C.c_int, [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(_P)]),
    ("vox_free", None, [_P]),
    ("vox_dim", C.c_int, [_P]),
    ("vox_plan_stats", C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                 C.POINTER(C.c_int64), C.POINTER(C.c_int)]),
    ("vox_feat_dim", C.c_int, [_P]),
    ("vox_expand_dim", C.c_int, [_P]),
    ("vox_precision", C.c_int, [_P]),
    ("vox_embed", C.c_int, [_P, _F, C.c_int, C.c_int, C.c_int, _F]),
    ("vox_embed_device", C.c_int, [_P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, _P]),
    ("vox_embed_utt", C.c_int, [_P, _F, C.c_int, C.c_int, _F]),
    ("vox_embed_device_lens", C.c_int,
     [_P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, _P]),
    ("vox_embed_lens", C.c_int, [_P, _F, C.c_int, C.c_int, C.c_int, C.c_void_p, _F]),
    ("vox_profile", C.c_int, [_P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _F,
                              C.POINTER(C.c_double), C.POINTER(C.c_double),
                              C.POINTER(C.c_int), C.c_int, _P]),
    ("vox_plan_describe", C.c_int, [_P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                    C.c_size_t]),
    ("vox_stats_pool_device", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, _P]),
    ("vox_asnorm_stats", C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                   C.c_void_p, C.c_void_p, C.c_void_p]),
    ("vox_last_error", C.c_char_p, []),
    ("vox_debug_taps", C.c_int, [_P, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                 C.POINTER(Tap), C.c_int, C.POINTER(C.c_int)]),
    ("vox_debug_run_ops", C.c_int, [_P, C.c_int, C.c_int, _P]),
    ("vox_debug_read", C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
    ("vox_debug_struct_size", C.c_int64, [C.c_int]),
    ("vox_sliding_cmn", C.c_int, [_F, C.c_int, C.c_int, C.c_int, C.c_int, _F]),
    ("vox_mat_shape", C.c_int, [C.c_char_p, C.c_int64, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("vox_read_mat", C.c_int, [C.c_char_p, C.c_int64, _F, C.c_int, C.c_int]),
    ("vox_parse_mat", C.c_int, [C.c_char_p, C.c_size_t, _F, C.c_int, C.c_int,
                                C.POINTER(C.c_size_t)]),
    ("vox_read_mat_kaldi", C.c_int, [C.c_char_p, C.c_int64, _F, C.c_int, C.c_int]),
    ("vox_mat_shapes", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]),
    ("vox_read_chunks", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                  C.c_int]),
    ("vox_read_chunks_ragged", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_void_p, C.c_int]),
    ("vox_parse_mat_kaldi", C.c_int, [C.c_char_p, C.c_size_t, _F, C.c_int, C.c_int,
                                      C.POINTER(C.c_size_t)]),
    ("vox_parse_mat_shape", C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(C.c_int),
                                      C.POINTER(C.c_int)]),
    ("vox_fbank_default_opts", None, [_FO]),
    ("vox_fbank_num_frames", C.c_int64, [C.c_int64, _FO]),
    ("vox_fbank_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int64, _FO,
                                   C.c_void_p, C.c_void_p]),
    ("vox_fbank_device_keyed", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                         C.c_int64, _FO, C.c_void_p, C.c_void_p]),
    ("vox_cm_blob_bytes", C.c_int64, [C.c_int, C.c_int]),
    ("vox_cm_compress_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p]),
    ("vox_sliding_cmn_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                                         C.c_int, C.c_void_p, C.c_void_p]),
    ("vox_cm_chunks_device", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int64, C.c_int,
                                       C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                       C.c_void_p]),
    ("vox_mat_kinds", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int]),
    ("vox_read_cm_payloads", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                       C.c_void_p, C.c_int]),
    ("vox_format_vec_flt", C.c_int64, [C.c_char_p, _F, C.c_int, C.c_void_p, C.c_size_t,
                                       C.POINTER(C.c_int64)]),
]
EXPORTED = [s[0] for s in _SIGS]


class NativeUnavailable(RuntimeError):
    pass


class VoxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libvoxemb error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load (once) and return the ctypes library; raise loudly if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeUnavailable(
            f"{LIB_PATH} not found -- build it with `python -m "
            "voxsrc2020_speaker_verification_amd.build_native` (there is no CPU fallback)")
    try:
        h = C.CDLL(LIB_PATH)
    except OSError as e:
        raise NativeUnavailable(f"cannot load {LIB_PATH}: {e}") from e
    for name, res, args in _SIGS:
        # an older build loaded for an A/B (tools/ab_libs.sh, VOXEMB_LIB) may lack
        # entry points added since; the product library must have them all
        if "VOXEMB_LIB" in os.environ and not hasattr(h, name):
            continue
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    _lib = h
    return h


def check(rc):
    """Raise VoxError for a negative status; return rc otherwise."""
    if rc < 0:
        msg = lib().vox_last_error()
        raise VoxError(rc, msg.decode() if msg else "")
    return rc


def fptr(a):
    return a.ctypes.data_as(_F)
