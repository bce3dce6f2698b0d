"""Python mirror of the reference's model-session interface.

The reference (tensorflow/tf_extract.py:75-111) imports a frozen graph and
calls `sess.run(outputs, {inputs: x})` once per <=1000-frame chunk of each
utterance.  `Extractor` is that session: it loads a weight blob into
libvoxemb on one HIP device and exposes

  * `run(x)`        -- one batch [N,T,F] (host numpy) -> [N,D]   (sess.run)
  * `run_device(...)` -- device-resident in/out (torch tensors)
  * `embed_utterance(feat)` -- the chunk rule + length-weighted average
                               (tf_extract.py:96-111), with the reference's
                               failure for T < 25 (ZeroDivisionError).

All compute is in the HIP library; there is no CPU fallback.
"""

from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _native
from ._native import check, fptr, lib

MAX_FRAMES = 1000  # tf_extract.py:96
MIN_FRAMES = 25    # tf_extract.py:101-102


def chunk_plan(T, max_frames=MAX_FRAMES):
    """[(start, length)] per tf_extract.py:102-107 (empty for T < 25)."""
    n = 1 + (T - 25) // max_frames
    out = []
    for i in range(max(n, 0)):
        L = max_frames if (i + 1) * max_frames <= T else T - i * max_frames
        out.append((i * max_frames, L))
    return out


class Extractor:
    def __init__(self, weights, device=0, precision="bf16"):
        prec = {"fp32": _native.VOX_FP32, "bf16": _native.VOX_BF16}[precision]
        h = C.c_void_p()
        L = lib()
        if isinstance(weights, (bytes, bytearray)):
            buf = C.create_string_buffer(bytes(weights), len(weights))
            check(L.vox_load_blob(buf, len(weights), int(device), prec, C.byref(h)))
        else:
            check(L.vox_load(os.fsencode(weights), int(device), prec, C.byref(h)))
        self._h = h
        self.device = int(device)
        self.precision = precision
        self.dim = check(L.vox_dim(h))
        self.feat_dim = check(L.vox_feat_dim(h))
        self.expand_dim = check(L.vox_expand_dim(h))

    def close(self):
        if getattr(self, "_h", None):
            lib().vox_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def plan_stats(self):
        """{built, hits, dropped, resident}: the native plan residency counters
        (vox_plan_stats)."""
        b, h, d, r = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
        check(lib().vox_plan_stats(self._h, C.byref(b), C.byref(h), C.byref(d), C.byref(r)))
        return {"built": b.value, "hits": h.value, "dropped": d.value, "resident": r.value}

    # -- sess.run ---------------------------------------------------------
    def run(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 3:
            raise ValueError("expected [N, T, F] features")
        n, t, f = x.shape
        out = np.empty((n, self.dim), np.float32)
        check(lib().vox_embed(self._h, fptr(x), n, t, f, fptr(out)))
        return out

    def run_device(self, x, out=None, stream=None):
        """x: contiguous float32 torch tensor [N,T,F] on this device.  Returns
        (or fills) a float32 [N,D] device tensor.  Launches on `stream`
        (torch.cuda.Stream or raw handle) -- the current torch stream by default."""
        import torch
        if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 3:
            raise ValueError("expected a contiguous float32 [N,T,F] device tensor")
        n, t, f = x.shape
        if out is None:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=x.device)
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        with self._ordered(stream, x.device) as sh:
            check(lib().vox_embed_device(self._h, C.c_void_p(x.data_ptr()), n, t, f,
                                         C.c_void_p(out.data_ptr()), C.c_void_p(sh)))
        return out

    def run_lens(self, x, lens):
        """Ragged batch (host numpy): x [N,T,F] with utterance i's lens[i]
        frames first and padding after (its values are ignored) -> [N,D], each
        row equal to run() on that utterance alone at T = lens[i]
        (vox_embed_lens; res2net bf16 plans)."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        if x.ndim != 3:
            raise ValueError("expected [N, T, F] features")
        n, t, f = x.shape
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        if lens.shape != (n,):
            raise ValueError("one length per utterance")
        out = np.empty((n, self.dim), np.float32)
        check(lib().vox_embed_lens(self._h, fptr(x), n, t, f, lens.ctypes.data, fptr(out)))
        return out

    def supports_lengths(self):
        """Whether this handle's plans take ragged batches (run_lens): probed
        once with a two-utterance batch (res2net bf16 plans do)."""
        if "_rag_ok" not in self.__dict__:
            try:
                x = np.zeros((2, 64, self.feat_dim), np.float32)
                self.run_lens(x, [64, 40])
                self._rag_ok = True
            except _native.VoxError:
                self._rag_ok = False
        return self._rag_ok

    def run_device_lens(self, x, lens, out=None, stream=None):
        """run_device for a ragged batch: lens is an int32 device tensor [N]
        (each in [1, T]; not checked on the device)."""
        import torch
        if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 3:
            raise ValueError("expected a contiguous float32 [N,T,F] device tensor")
        n, t, f = x.shape
        if lens.dtype != torch.int32 or lens.shape != (n,) or lens.device != x.device:
            raise ValueError("expected an int32 [N] lengths tensor on the input's device")
        if out is None:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=x.device)
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        with self._ordered(stream, x.device) as sh:
            check(lib().vox_embed_device_lens(self._h, C.c_void_p(x.data_ptr()), n, t, f,
                                              C.c_void_p(lens.data_ptr()),
                                              C.c_void_p(out.data_ptr()), C.c_void_p(sh)))
        return out

    def _ordered(self, stream, device):
        """Context giving the raw handle to launch on for a torch stream (or raw
        handle).  The legacy default stream has handle 0, which the C-ABI reads
        as "the model's own stream" (non-blocking: NOT ordered with the default
        stream, so the kernels could read an input copy still in flight and the
        caller could read the output before they finish -- found on a staged
        batch, DESIGN.md "Streams").  For it the launch goes to a side stream
        fenced both ways with the caller's stream."""
        import contextlib
        import torch
        sh = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        if sh:
            return contextlib.nullcontext(sh)
        caller = stream if hasattr(stream, "wait_stream") else torch.cuda.default_stream(device)
        side = self.__dict__.get("_side")
        if side is None or side.device != caller.device:
            side = self._side = torch.cuda.Stream(caller.device)

        @contextlib.contextmanager
        def fenced():
            side.wait_stream(caller)
            yield side.cuda_stream
            caller.wait_stream(side)
        return fenced()

    def run_device_staged(self, x, stream=None):
        """run_device through input/output buffers kept per batch shape: the
        native plan (and its captured hipGraph) is keyed on the device
        pointers, so feeding freshly allocated tensors every batch rebuilds and
        re-captures it each time; here same-shape batches replay one graph
        (one device-to-device copy of the input per batch).  Returns the
        staged output tensor, valid until the next call with this shape."""
        import torch
        if x.dtype != torch.float32 or x.dim() != 3:
            raise ValueError("expected a float32 [N,T,F] device tensor")
        stage = self.__dict__.setdefault("_stage", {})
        key = (tuple(x.shape), x.device)
        if key not in stage:
            if len(stage) >= 4:   # a few shapes (the bucketed chunk lengths)
                stage.pop(next(iter(stage)))
            stage[key] = (torch.empty(x.shape, dtype=torch.float32, device=x.device),
                          torch.empty((x.shape[0], self.dim), dtype=torch.float32, device=x.device))
        xs, out = stage[key]
        xs.copy_(x)
        return self.run_device(xs, out, stream)

    def profile(self, x, reps=5, stream=None, max_ops=4096):
        """Per-op timing of one forward (HIP events around each launch)."""
        import torch
        n, t, f = x.shape
        ms = np.zeros(max_ops, np.float32)
        fl = np.zeros(max_ops, np.float64)
        by = np.zeros(max_ops, np.float64)
        kind = np.zeros(max_ops, np.int32)
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        with self._ordered(stream, x.device) as sh:
            nops = check(lib().vox_profile(
                self._h, C.c_void_p(x.data_ptr()), n, t, f, int(reps), fptr(ms),
                fl.ctypes.data_as(C.POINTER(C.c_double)), by.ctypes.data_as(C.POINTER(C.c_double)),
                kind.ctypes.data_as(C.POINTER(C.c_int)), max_ops, C.c_void_p(sh)))
        return dict(ms=ms[:nops], flops=fl[:nops], bytes=by[:nops], kind=kind[:nops])

    def describe(self, x):
        """One line per kernel launch of the plan for x's shape."""
        n, t, f = x.shape
        need = check(lib().vox_plan_describe(self._h, C.c_void_p(x.data_ptr()), n, t, f, None, 0))
        buf = C.create_string_buffer(need)
        check(lib().vox_plan_describe(self._h, C.c_void_p(x.data_ptr()), n, t, f, buf, need))
        return buf.value.decode().strip().split("\n")

    # -- layer-by-layer parity support (tests) ------------------------------
    def layer_outputs(self, x, utts=None):
        """Run the plan for the device batch x ([N,T,F] float32 torch tensor)
        launch by launch and return (taps, embeddings): taps[i] is the output
        of oracle layer i (oracle/models_ref.py `layers`) as a float32 numpy
        array [n,h,w,c], read right after the launch that completes it.
        utts: read only these utterances' rows of every tap ([len(utts),h,w,c];
        the whole batch still runs -- for the big-batch plans)."""
        import torch
        n, t, f = x.shape
        out = torch.empty((n, self.dim), dtype=torch.float32, device=x.device)
        L = lib()
        xp, op = C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr())
        nops = C.c_int()
        nt = check(L.vox_debug_taps(self._h, xp, n, t, f, op, None, 0, C.byref(nops)))
        taps = (_native.Tap * max(nt, 1))()
        check(L.vox_debug_taps(self._h, xp, n, t, f, op, taps, nt, C.byref(nops)))
        torch.cuda.synchronize(x.device)
        res, begin = [], 0
        for tp in taps[:nt]:
            check(L.vox_debug_run_ops(self._h, begin, tp.op_end, None))
            begin = tp.op_end
            es = 2 if tp.dtype == _native.VOX_BF16 else 4
            sel = list(range(tp.n)) if utts is None else [int(u) for u in utts]
            per = tp.h * tp.w * tp.ld * es          # bytes of one utterance's rows
            raw = np.empty((len(sel), tp.h * tp.w, tp.ld * es), np.uint8)
            if utts is None:
                check(L.vox_debug_read(raw.ctypes.data_as(C.c_void_p), C.c_void_p(tp.data), raw.nbytes))
            else:
                for j, u in enumerate(sel):
                    if not 0 <= u < tp.n:
                        raise IndexError(f"utterance {u} outside the batch of {tp.n}")
                    check(L.vox_debug_read(raw[j].ctypes.data_as(C.c_void_p),
                                           C.c_void_p(tp.data + u * per), per))
            raw = raw.reshape(len(sel) * tp.h * tp.w, tp.ld * es)
            if es == 2:
                a = (raw.view(np.uint16)[:, :tp.c].astype(np.uint32) << 16).view(np.float32)
            else:
                a = raw.view(np.float32)[:, :tp.c].copy()
            res.append(a.reshape(len(sel), tp.h, tp.w, tp.c))
        # the rest of the plan: pooling + head
        check(L.vox_debug_run_ops(self._h, begin, nops.value, None))
        return res, out.cpu().numpy()

    # -- tf_extract chunk loop ---------------------------------------------
    def embed_utterance(self, feat):
        feat = np.ascontiguousarray(feat, dtype=np.float32)
        T, f = feat.shape
        if T < MIN_FRAMES:
            # the reference divides 0 by 0 here (tf_extract.py:111)
            raise ZeroDivisionError(f"utterance has {T} < {MIN_FRAMES} frames")
        out = np.empty(self.dim, np.float32)
        check(lib().vox_embed_utt(self._h, fptr(feat), T, f, fptr(out)))
        return out
