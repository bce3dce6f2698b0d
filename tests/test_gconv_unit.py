"""The row-streamed grouped 3x3 conv (gconv.hip, DPN68's cardinality-32
bn_relu_conv, dpn_model.py:40-45,49) on random data against a numpy
emulation with the same bf16 rounding points: prologue relu((x-m)*inv)
rounded to bf16, TF SAME zero padding AFTER the activation (stride 2:
pad-begin = pad_total // 2, models.py conv2d / dpn_model.py:43-44), bf16
weights, fp32 accumulation, bf16 output.  The expanded weight layout is
rebuilt here from its definition in api.cpp (make_conv, `wgc`).  Called through
the internal launcher (C++ symbol).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bf16(a):
    a = np.ascontiguousarray(a, np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32)


class GconvParams(C.Structure):
    _fields_ = [("x", C.c_void_p), ("ldx", C.c_int),
                ("in_mean", C.c_void_p), ("in_inv", C.c_void_p),
                ("w", C.c_void_p), ("y", C.c_void_p), ("ldy", C.c_int),
                ("N", C.c_int), ("H", C.c_int), ("W", C.c_int), ("C", C.c_int),
                ("Ho", C.c_int), ("Wo", C.c_int), ("gw", C.c_int),
                ("sh", C.c_int), ("ph", C.c_int), ("pw", C.c_int),
                ("seg", C.c_int), ("nseg", C.c_int), ("rs_force", C.c_int)]


def tf_same(n, s, k=3):
    o = (n + s - 1) // s
    tot = max((o - 1) * s + k - n, 0)
    return o, tot // 2, tot - tot // 2


def expand(k, gw):
    """HWIO grouped kernel [3,3,gw,C] -> [C/16][NM][64][8] (api.cpp make_conv)."""
    Cc = k.shape[3]
    NM = 9 if gw == 32 else 5
    out = np.zeros((Cc // 16, NM, 64, 8), np.float32)
    kt = k.reshape(9, gw, Cc)
    for sg in range(Cc // 16):
        for m in range(NM):
            for l in range(64):
                co, q = 16 * sg + (l & 15), l >> 4
                for e in range(8):
                    if gw == 32:
                        tap, ci = m, 32 * (co // 32) + 8 * q + e
                    else:
                        tap, ci = 2 * m + (q >> 1), 16 * sg + 8 * (q & 1) + e
                    if tap < 9 and ci // gw == co // gw:
                        out[sg, m, l, e] = kt[tap, ci % gw, co]
    return out


def reference(X, k, m, inv, gw, s):
    N, H, W, Cc = X.shape
    Ho, pt, pb = tf_same(H, s)
    Wo, pl, pr = tf_same(W, s)
    a = bf16(np.maximum((X - m) * inv, 0))
    a = np.pad(a, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    G = Cc // gw
    out = np.zeros((N, Ho, Wo, Cc), np.float32)
    for ky in range(3):
        for kx in range(3):
            win = a[:, ky:ky + s * (Ho - 1) + 1:s, kx:kx + s * (Wo - 1) + 1:s]
            win = win.reshape(N, Ho, Wo, G, gw)
            kk = k[ky, kx].reshape(gw, G, gw)          # [ci][g][co]
            out += np.einsum("nhwgc,cgd->nhwgd", win, kk).reshape(N, Ho, Wo, Cc)
    return bf16(out), pt, pl


def run(N, H, W, Cc, gw, s, nseg, seed):
    import torch
    from voxsrc2020_speaker_verification_amd import _native
    rng = np.random.default_rng(seed)
    X = bf16(rng.standard_normal((N, H, W, Cc)))
    k = bf16(rng.standard_normal((3, 3, gw, Cc)) / np.sqrt(9 * gw))
    m = (rng.standard_normal(Cc) * 0.3).astype(np.float32)
    inv = (0.5 + rng.random(Cc)).astype(np.float32)
    ref, pt, pl = reference(X, k, m, inv, gw, s)
    Ho, Wo = ref.shape[1:3]
    tb = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda().to(torch.bfloat16)
    tf = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    xd, wd, md, vd = tb(X), tb(expand(k, gw)), tf(m), tf(inv)
    yd = torch.full((N, Ho, Wo, Cc), float("nan"), dtype=torch.bfloat16, device="cuda")
    p = GconvParams()
    p.x, p.ldx, p.in_mean, p.in_inv = xd.data_ptr(), Cc, md.data_ptr(), vd.data_ptr()
    p.w, p.y, p.ldy = wd.data_ptr(), yd.data_ptr(), Cc
    p.N, p.H, p.W, p.C, p.Ho, p.Wo, p.gw = N, H, W, Cc, Ho, Wo, gw
    p.sh, p.ph, p.pw = s, pt, pl
    p.seg = (Ho + nseg - 1) // nseg
    p.nseg = (Ho + p.seg - 1) // p.seg
    fn = getattr(_native.lib(), "_ZN3vox12launch_gconvERKNS_11GconvParamsEP12ihipStream_t")
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(GconvParams), C.c_void_p]
    assert fn(C.byref(p), None) == 0
    torch.cuda.synchronize()
    return yd.float().cpu().numpy(), ref


@pytest.mark.parametrize("N,H,W,Cc,gw,s,nseg", [
    (2, 37, 80, 128, 4, 1, 3),     # stage 1 (RS 1)
    (1, 30, 80, 256, 8, 2, 1),     # stage 2 block 0: even H, pads (0,1)
    (2, 31, 80, 256, 8, 2, 2),     # odd H: pads (1,1) on rows
    (2, 23, 40, 256, 8, 1, 2),     # stage 2 (RS 2)
    (2, 19, 20, 512, 16, 1, 1),    # stage 3 (RS 4)
    (1, 33, 40, 512, 16, 2, 3),    # stage 3 block 0
    (2, 21, 10, 1024, 32, 1, 2),   # stage 4 (RS 8, gw 32)
    (1, 41, 20, 1024, 32, 2, 2),   # stage 4 block 0
    (1, 5, 40, 128, 4, 1, 1),      # fewer rows than one window
    (1, 7, 80, 128, 4, 1, 3),      # segments of 3, 3, 1 steps (the two-step prefetch's ends)
    (2, 2, 80, 256, 8, 1, 1),      # a single step
    (1, 9, 20, 512, 16, 1, 2),     # RS 4: a segment with one partial step
])
def test_gconv_matches_emulation(N, H, W, Cc, gw, s, nseg):
    got, ref = run(N, H, W, Cc, gw, s, nseg, seed=H * 7 + gw)
    d = np.abs(got - ref)
    assert np.isfinite(got).all()
    assert np.mean(d == 0) >= 0.99, f"only {np.mean(d == 0):.4f} exact"
    assert d.max() <= 2.0 ** -6 * np.abs(ref).max(), f"max diff {d.max()}"
