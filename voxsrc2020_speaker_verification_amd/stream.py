"""Streaming extraction of a Kaldi feature scp with bounded host memory.

The reference (tensorflow/tf_extract.py:85-113) streams: a reader process
decodes one utterance at a time through the `apply-cmvn-sliding` pipe (:63)
into a Queue(32), and the session runs each <= 1000-frame chunk on its own
(:96-108).  Here the same results come out of three stages that overlap:

  1. planning (headers only): every utterance's frame count from its matrix
     header (`vox_mat_shapes`), the chunk rule (:96-107) applied over the whole
     shard (one planning window).  Ragged mode (res2net bf16, the default where
     the plan supports it): the chunks sorted by length and cut into full
     batches padded to a coarse length grid (padded_length), each chunk's
     frame count passed to the kernels (vox_embed_device_lens) -- real length
     distributions give full batches and resident plans; exact mode: equal-
     length chunks batched together.  Either way a chunk's embedding is the
     bits of its own unpadded run (batch independence, tests/test_ragged.py);
  2. reading: each batch's chunks decoded, CMN'd and sliced straight into a
     pinned host buffer by the native reader (`vox_read_chunks`, host threads)
     while the lane's previous batch runs on the GPU;
  3. compute: the batches go round-robin to `lanes` extraction handles, each
     driven by its own host thread with its own streams, device buffers and
     resident plans; a batch's H2D copy is queued on the lane's copy stream
     (overlapping the previous forward), its forward and D2H copy on the
     lane's compute stream.

Host memory is two batches of features per lane plus one embedding per
utterance; nothing grows with the features of the shard.  The per-utterance
combination (length-weighted mean, :108-111) is the float32 arithmetic of
`extract.embed_utterances`, so the arks are byte-identical to it.
"""

from __future__ import annotations

import ctypes as C
import os
import threading
import time

import numpy as np

from ._native import check, lib
from .extractor import MAX_FRAMES, MIN_FRAMES, chunk_plan
from .kaldi import CMN_WINDOW, parse_rxfile


def default_threads():
    """Host threads for the reader: the CPUs this process may use (affinity,
    capped by a cgroup CPU quota), at most 16."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, min(16, n))


class ChunkTable:
    """The utterances of an scp (list of (key, rxfile)) with their frame
    ranges, read from the matrix headers only."""

    def __init__(self, entries, threads=None):
        self.threads = threads or default_threads()
        self.keys = [k for k, _ in entries]
        n = len(entries)
        self._paths = []
        offs = np.zeros(n, np.int64)
        rngs = []
        for i, (_, rx) in enumerate(entries):
            path, off, rng = parse_rxfile(rx)
            self._paths.append(os.fsencode(path))
            offs[i] = off
            rngs.append(rng)
        self._path_arr = (C.c_char_p * max(n, 1))(*self._paths)
        self.offsets = offs
        rows = np.zeros(n, np.int32)
        cols = np.zeros(n, np.int32)
        if n:
            check(lib().vox_mat_shapes(self._path_arr, offs.ctypes.data, n, rows.ctypes.data,
                                       cols.ctypes.data, self.threads))
        # the rxfile's [r0:r1,c0:c1] range (kaldi.parse_rxfile), as numpy slicing reads it
        self.r0 = np.zeros(n, np.int32)
        self.T = rows.copy()
        self.c0 = np.zeros(n, np.int32)
        self.F = cols.copy()
        for i, rng in enumerate(rngs):
            if rng is None:
                continue
            rs, cs = (rng + (slice(None),))[:2]
            r0, r1, _ = rs.indices(int(rows[i]))
            c0, c1, _ = cs.indices(int(cols[i]))
            self.r0[i], self.T[i] = r0, max(0, r1 - r0)
            self.c0[i], self.F[i] = c0, max(0, c1 - c0)
        if n and (self.F != self.F[0]).any():
            raise ValueError("utterances with different feature dimensions in one scp")
        self.feat_dim = int(self.F[0]) if n else 0
        self._rows, self._cols = rows, cols
        self._cm_ok = None

    def __len__(self):
        return len(self.keys)

    def read(self, items, L, out, cmn=True, threads=None):
        """Chunks [(u, ci, start)] of length L -> out ([>= n*L*F] float32, numpy
        array or torch tensor in host memory)."""
        n = len(items)
        u = np.fromiter((it[0] for it in items), np.int64, n)
        st = np.fromiter((it[2] for it in items), np.int32, n)
        paths = (C.c_char_p * n)(*[self._paths[i] for i in u])
        offs = np.ascontiguousarray(self.offsets[u])
        r0 = np.ascontiguousarray(self.r0[u])
        T = np.ascontiguousarray(self.T[u])
        c0 = np.ascontiguousarray(self.c0[u])
        ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
        check(lib().vox_read_chunks(paths, offs.ctypes.data, r0.ctypes.data, T.ctypes.data,
                                    c0.ctypes.data, st.ctypes.data, n, self.feat_dim, int(L),
                                    CMN_WINDOW if cmn else 0, C.c_void_p(ptr),
                                    threads or self.threads))

    def cm_device_ok(self):
        """Every matrix a whole "CM " one (no [range]): the device reader
        (vox_cm_chunks_device) can decode it."""
        if self._cm_ok is None:
            n = len(self)
            kinds = np.zeros(n, np.int32)
            if n:
                check(lib().vox_mat_kinds(self._path_arr, self.offsets.ctypes.data, n,
                                          kinds.ctypes.data, self.threads))
            self._cm_ok = bool(n) and bool(
                (kinds == 2).all() and (self.r0 == 0).all() and (self.c0 == 0).all() and
                (self.T == self._rows).all() and (self.F == self._cols).all() and (self.T > 8).all())
        return self._cm_ok

    def cm_batch(self, items, lens, cmn=True):
        """The device reader's plan of one batch: its utterances (first
        appearance order), their payload offsets and the rows each must decode
        (the CMN windows of the batch's chunks inside them) -> (utts, meta
        int64 [blob_off | frame_off | rows | item_utt | item_start | item_len],
        payload bytes, total rows, max rows)."""
        F = self.feat_dim
        slot, utts, hi = {}, [], []
        iu = np.empty(len(items), np.int64)
        for i, (u, _, st) in enumerate(items):
            k = slot.get(u)
            if k is None:
                k = slot[u] = len(utts)
                utts.append(u)
                hi.append(0)
            iu[i] = k
            hi[k] = max(hi[k], st + lens[i])
        U = len(utts)
        T = self.T[utts].astype(np.int64)
        hi = np.asarray(hi, np.int64)
        need = np.minimum(T, np.maximum(hi + CMN_WINDOW - CMN_WINDOW // 2, CMN_WINDOW)) if cmn else hi
        meta = np.empty(3 * U + 2 + 3 * len(items), np.int64)
        meta[0] = 0
        np.cumsum(16 + 8 * F + T * F, out=meta[1:U + 1])
        meta[U + 1] = 0
        np.cumsum(need, out=meta[U + 2:2 * U + 2])
        meta[2 * U + 2:3 * U + 2] = T
        n = len(items)
        meta[3 * U + 2:3 * U + 2 + n] = iu
        meta[3 * U + 2 + n:3 * U + 2 + 2 * n] = [it[2] for it in items]
        meta[3 * U + 2 + 2 * n:] = lens
        return utts, meta, int(meta[U]), int(meta[2 * U + 1]), int(need.max())

    def read_cm_payloads(self, utts, meta, buf, threads=None):
        """The "CM " payloads of `utts` into buf (pinned host memory) at the
        offsets cm_batch planned."""
        U = len(utts)
        paths = (C.c_char_p * U)(*[self._paths[u] for u in utts])
        offs = np.ascontiguousarray(self.offsets[utts])
        ptr = buf.data_ptr() if hasattr(buf, "data_ptr") else buf.ctypes.data
        check(lib().vox_read_cm_payloads(paths, offs.ctypes.data, U, meta.ctypes.data,
                                         self.feat_dim, C.c_void_p(ptr), threads or self.threads))

    def read_ragged(self, items, lens, stride, out, cmn=True, threads=None):
        """Chunks [(u, ci, start)] of lens[i] frames each into rows
        [i*stride, i*stride + lens[i]) of out (a ragged batch; the rows after
        each chunk are left as they are: padding)."""
        n = len(items)
        u = np.fromiter((it[0] for it in items), np.int64, n)
        st = np.fromiter((it[2] for it in items), np.int32, n)
        ln = np.ascontiguousarray(lens, dtype=np.int32)
        paths = (C.c_char_p * n)(*[self._paths[i] for i in u])
        offs = np.ascontiguousarray(self.offsets[u])
        r0 = np.ascontiguousarray(self.r0[u])
        T = np.ascontiguousarray(self.T[u])
        c0 = np.ascontiguousarray(self.c0[u])
        ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
        check(lib().vox_read_chunks_ragged(paths, offs.ctypes.data, r0.ctypes.data, T.ctypes.data,
                                           c0.ctypes.data, st.ctypes.data, ln.ctypes.data, n,
                                           self.feat_dim, int(stride), CMN_WINDOW if cmn else 0,
                                           C.c_void_p(ptr), threads or self.threads))


def padded_length(L, max_frames=MAX_FRAMES):
    """Row count a ragged batch whose longest chunk has L frames is padded to:
    a grid of ~1/16 steps (8 frames up to 128, 16 up to 256, 32 up to 512, 64
    beyond; the chunk maximum itself at the top), so batches of neighbouring
    lengths share a resident plan (and its graph) while padding stays a few
    per cent of the frames."""
    q = 8 if L <= 128 else 16 if L <= 256 else 32 if L <= 512 else 64
    Lp = -(-L // q) * q
    return min(Lp, max(L, max_frames))


def plan_batches(lengths, batch, keys=None, ragged=False):
    """The chunk rule over every utterance -> (per-utterance chunk plans,
    batches).  Exact mode: equal-length chunks bucketed, batches
    (L, [(u, ci, start), ...]) with scp order inside a bucket.  Ragged mode
    (vox_embed_lens): every chunk sorted by length, consecutive runs of `batch`
    chunks padded to padded_length(longest) -> (Lp, items, lens); a chunk's
    embedding is the same either way (bitwise: tests/test_ragged.py).
    Batches are ordered by size (frames) descending, so the first sizes the
    device workspace once.  An utterance shorter than 25 frames raises
    ZeroDivisionError, as tf_extract.py:111 does."""
    plans, buckets = [], {}
    for u, T in enumerate(lengths):
        plan = chunk_plan(int(T))
        if not plan:
            key = keys[u] if keys is not None else u
            raise ZeroDivisionError(f"utterance {key} has {int(T)} < {MIN_FRAMES} frames "
                                    "(tf_extract.py:102,111)")
        plans.append(plan)
        for ci, (s, L) in enumerate(plan):
            buckets.setdefault(L, []).append((u, ci, s))
    if ragged:
        chunks = [(L, it) for L in sorted(buckets, reverse=True) for it in buckets[L]]
        batches = []
        for b in range(0, len(chunks), batch):
            part = chunks[b:b + batch]
            batches.append((padded_length(part[0][0]), [it for _, it in part],
                            [L for L, _ in part]))
    else:
        batches = [(L, items[b:b + batch]) for L, items in buckets.items()
                   for b in range(0, len(items), batch)]
    batches.sort(key=lambda b: -b[0] * len(b[1]))
    return plans, batches


class Combiner:
    """Per-utterance length-weighted mean of its chunk embeddings in chunk
    order (extract.embed_utterances' float32 arithmetic, tf_extract.py:108-111:
    acc = 0; acc = acc + e_c * L_c; acc / sum L), a batch at a time in numpy:
    single-chunk utterances are finished with the batch; the rows of
    multi-chunk ones wait in one array and an utterance is finished, with the
    others of its chunk count, in the batch that brings its last chunk.  The
    operations are the scalar loop's, element-wise in float32, so the bits are
    the same."""

    def __init__(self, plans, dim):
        self.plans = plans
        self.out = np.empty((len(plans), dim), np.float32)
        self.done = 0
        nch = np.fromiter((len(p) for p in plans), np.int64, len(plans))
        self._nch = nch
        self._left = nch.copy()
        # rows of multi-chunk utterances: slot base[u] + ci
        multi = nch > 1
        base = np.full(len(plans), -1, np.int64)
        base[multi] = np.concatenate([[0], np.cumsum(nch[multi])[:-1]]) if multi.any() else []
        self._base = base
        self._pend = np.empty((int(nch[multi].sum()), dim), np.float32)
        kmax = int(nch.max()) if len(plans) else 1
        self._lens = np.zeros((len(plans), kmax), np.float32)     # chunk lengths
        for k, p in enumerate(plans):
            self._lens[k, :len(p)] = [L for _, L in p]
        self._tot = self._lens.sum(axis=1, keepdims=True)         # exact: integers < 2^24

    def add_batch(self, items, rows):
        """items [(u, ci, start)] of one batch, rows [n, dim] float32."""
        rows = np.asarray(rows, np.float32)
        uc = np.array([it[:2] for it in items], np.int64).reshape(-1, 2)
        u, ci = uc[:, 0], uc[:, 1]
        one = self._nch[u] == 1
        if one.all():
            L = self._lens[u, :1]
            self.out[u] = (np.float32(0) + rows * L) / L
            self.done += len(u)
            return
        if one.any():
            us = u[one]
            L = self._lens[us, :1]
            self.out[us] = (np.float32(0) + rows[one] * L) / L
            self.done += len(us)
        mu, mc = u[~one], ci[~one]
        self._pend[self._base[mu] + mc] = rows[~one]
        np.subtract.at(self._left, mu, 1)
        fin = np.unique(mu[self._left[mu] == 0])
        if not len(fin):
            return
        for k in np.unique(self._nch[fin]):
            us = fin[self._nch[fin] == k]
            lens, b0 = self._lens[us], self._base[us]
            acc = np.float32(0) + self._pend[b0] * lens[:, :1]
            for c in range(1, int(k)):
                acc = acc + self._pend[b0 + c] * lens[:, c:c + 1]
            self.out[us] = acc / self._tot[us]
            self.done += len(us)

    def add(self, u, ci, row):
        self.add_batch([(u, ci, 0)], np.asarray(row, np.float32)[None])


class SyncRunner:
    """Batches through a synchronous embed function (host numpy in and out):
    the CPU / test form of the pipeline."""

    def __init__(self, table, embed_batch, cmn=True):
        self.table, self.embed, self.cmn = table, embed_batch, cmn

    def run(self, batches):
        for bid, (L, items) in enumerate(batches):
            x = np.empty((len(items), L, self.table.feat_dim), np.float32)
            self.table.read(items, L, x, self.cmn)
            yield bid, self.embed(x)


class LanePool:
    """`lanes` extraction handles on one device, each driven by its own host
    thread: lane k takes batches k, k + K, k + 2K, ...; for each it reads the
    chunks into one of its two pinned buffers with the native reader on the
    lane's reader thread (the GIL is released in every native call, so reading,
    planning and launching run in parallel), queues the H2D on its copy stream
    (into one of two device buffers) and the forward + D2H on its compute
    stream, and then finishes its previous batch -- so every lane keeps two
    batches in flight, batch i + 1 is read while batch i is queued and batch
    i - 1 collected, and a batch's PCIe transfer overlaps the previous batch's
    forward."""

    def __init__(self, extractors, table, batches, cmn=True, device_reader=None):
        import torch
        self.torch = torch
        self.exs = list(extractors)
        self.table, self.cmn = table, cmn
        self.dev = torch.device("cuda", self.exs[0].device)
        F, dim, K = table.feat_dim, self.exs[0].dim, len(self.exs)
        max_el = max((len(b[1]) * b[0] * F for b in batches), default=1)
        max_n = max((len(b[1]) for b in batches), default=1)
        # ragged batches (L, items, lens): per-lane device lengths + pinned copies
        self.ragged = bool(batches) and len(batches[0]) == 3
        # device reader (whole "CM " matrices, opt-in): the payload bytes cross
        # PCIe and the GPU decodes, CMNs and gathers the chunks
        # (vox_cm_chunks_device) -- a quarter of the float32 bytes and about one
        # host thread instead of the reader's pool, at about the host reader's
        # extraction rate (its CMN is a serial chain per (utterance, bin):
        # DESIGN.md "Device reader")
        if device_reader and not (bool(batches) and table.cm_device_ok()):
            raise ValueError("the device reader needs whole \"CM \" matrices (no [range])")
        self.devread = bool(device_reader)
        if self.devread:
            mb = mm = mr = 1
            for b in batches:
                _, meta, nbytes, total, _ = table.cm_batch(b[1], self._lens(b), cmn)
                mb, mm, mr = max(mb, nbytes), max(mm, len(meta)), max(mr, total)
            self.h_blob = [[torch.empty(mb, dtype=torch.uint8).pin_memory() for _ in range(2)]
                           for _ in range(K)]
            self.h_meta = [[torch.empty(mm, dtype=torch.int64).pin_memory() for _ in range(2)]
                           for _ in range(K)]
            self.d_blob = [[torch.empty(mb, dtype=torch.uint8, device=self.dev) for _ in range(2)]
                           for _ in range(K)]
            self.d_meta = [[torch.empty(mm, dtype=torch.int64, device=self.dev) for _ in range(2)]
                           for _ in range(K)]
            self.d_work = [torch.empty(2 * mr * F, dtype=torch.float32, device=self.dev)
                           for _ in range(K)]
            self.slot_info = [[None, None] for _ in range(K)]
        self.d_len = [[torch.empty(max_n, dtype=torch.int32, device=self.dev) for _ in range(2)]
                      for _ in range(K)]
        self.h_len = [[torch.empty(max_n, dtype=torch.int32).pin_memory() for _ in range(2)]
                      for _ in range(K)]
        self.threads = max(1, table.threads // K)
        self.streams = [torch.cuda.Stream(self.dev) for _ in range(K)]
        # H2D copies on a stream of their own per lane, into two staging buffers,
        # so batch i+1's features cross PCIe while batch i computes (a fast
        # model -- the TDNN at ~1e8 frames/s -- reads ~30 GB/s of float32
        # features; the device reader's decode / CMN / gather kernels run there
        # too); the compute stream moves a batch from its staging buffer into
        # the lane's one input buffer (a D2D copy, microseconds), so the
        # resident plans, keyed on the input address, stay one per shape
        self.copy_streams = [torch.cuda.Stream(self.dev) for _ in range(K)]
        stage = 0 if self.devread else max_el    # host float32 staging (host reader only)
        self.d_stage = [[torch.empty(max_el, dtype=torch.float32, device=self.dev)
                         for _ in range(2)] for _ in range(K)]
        self.d_in = [torch.empty(max_el, dtype=torch.float32, device=self.dev) for _ in range(K)]
        self.d_out = [torch.empty(max_n * dim, dtype=torch.float32, device=self.dev) for _ in range(K)]
        self.h_in = [[torch.empty(stage, dtype=torch.float32).pin_memory() for _ in range(2)]
                     for _ in range(K)]
        self.h_out = [[torch.empty(max_n * dim, dtype=torch.float32).pin_memory() for _ in range(2)]
                      for _ in range(K)]
        # host seconds per phase, summed over the lanes (tools/bench_extract.py)
        self.phase = {"read": 0.0, "launch": 0.0, "wait": 0.0}
        self._lock = threading.Lock()

    @staticmethod
    def _lens(batch):
        return batch[2] if len(batch) == 3 else [batch[0]] * len(batch[1])

    def _read(self, k, j, batch, free_ev):
        """Batch `batch` into lane k's pinned buffers j (the lane's reader thread)
        once the H2D that last read them (free_ev) is done."""
        if free_ev is not None:
            free_ev.synchronize()
        L, items = batch[0], batch[1]
        if self.ragged:
            self.h_len[k][j][:len(items)].copy_(self.torch.tensor(batch[2], dtype=self.torch.int32))
        if self.devread:
            utts, meta, nbytes, total, mx = self.table.cm_batch(items, self._lens(batch), self.cmn)
            self.h_meta[k][j][:len(meta)].copy_(self.torch.from_numpy(meta))
            self.table.read_cm_payloads(utts, meta, self.h_blob[k][j], self.threads)
            self.slot_info[k][j] = (len(utts), len(meta), nbytes, total, mx)
            return
        hin = self.h_in[k][j]
        if self.ragged:
            self.table.read_ragged(items, batch[2], L, hin, self.cmn, self.threads)
        else:
            self.table.read(items, L, hin, self.cmn, self.threads)

    def _lane(self, k, batches, results, stop):
        from concurrent.futures import ThreadPoolExecutor
        torch, ex, s, cs = self.torch, self.exs[k], self.streams[k], self.copy_streams[k]
        F, dim = self.table.feat_dim, ex.dim
        mine = list(range(k, len(batches), len(self.exs)))
        prev = None              # (bid, n, done event, pinned output)
        free = [None, None]      # event after the H2D that last read h_in[k][j]
        used = [None, None]      # event after the forward that last read d_stage / d_len[k][j]
        clock, ph = time.perf_counter, {"read": 0.0, "launch": 0.0, "wait": 0.0}
        # the lane's reader thread reads batch i + 1 (native, GIL released) while
        # this thread queues batch i and collects batch i - 1
        reader = ThreadPoolExecutor(1)
        fut = None
        try:
            torch.cuda.set_device(self.dev)
            if mine:
                fut = reader.submit(self._read, k, 0, batches[mine[0]], None)
            for i, b in enumerate(mine):
                if stop:
                    return
                L, items = batches[b][0], batches[b][1]
                n, j = len(items), i & 1
                t1 = clock()
                fut.result()                      # batch b is in h_in[k][j]
                fut = None
                t2 = clock()
                hin, hl = self.h_in[k][j], self.h_len[k][j]
                xs, x = self.d_stage[k][j][:n * L * F], self.d_in[k][:n * L * F]
                o, dl = self.d_out[k][:n * dim], self.d_len[k][j][:n]
                with torch.cuda.stream(cs):
                    if used[j] is not None:
                        cs.wait_event(used[j])
                    if self.devread:
                        # payload bytes over PCIe, then decode + CMN + gather into
                        # the staging buffer -- on the copy stream, beside the
                        # previous batch's forward
                        U, nm, nbytes, total, mx = self.slot_info[k][j]
                        self.d_blob[k][j][:nbytes].copy_(self.h_blob[k][j][:nbytes], non_blocking=True)
                        self.d_meta[k][j][:nm].copy_(self.h_meta[k][j][:nm], non_blocking=True)
                        check(lib().vox_cm_chunks_device(
                            C.c_void_p(self.d_blob[k][j].data_ptr()),
                            C.c_void_p(self.d_meta[k][j].data_ptr()), U, total, mx, n, L, F,
                            CMN_WINDOW if self.cmn else 0, C.c_void_p(self.d_work[k].data_ptr()),
                            C.c_void_p(xs.data_ptr()), C.c_void_p(cs.cuda_stream)))
                    else:
                        xs.copy_(hin[:n * L * F], non_blocking=True)
                    if self.ragged:
                        dl.copy_(hl[:n], non_blocking=True)
                    free[j] = torch.cuda.Event()
                    free[j].record(cs)
                if i + 1 < len(mine):
                    fut = reader.submit(self._read, k, j ^ 1, batches[mine[i + 1]], free[j ^ 1])
                s.wait_event(free[j])
                with torch.cuda.stream(s):
                    x.copy_(xs)
                if self.ragged:
                    ex.run_device_lens(x.view(n, L, F), dl, o.view(n, dim), s)
                else:
                    ex.run_device(x.view(n, L, F), o.view(n, dim), s)
                h = self.h_out[k][j]
                with torch.cuda.stream(s):
                    # after the forward, which also reads d_len[k][j] (copied into
                    # the plan's workspace on s): the copy stream may refill both
                    used[j] = torch.cuda.Event()
                    used[j].record(s)
                    h[:n * dim].copy_(o, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(s)
                t3 = clock()
                if prev is not None:
                    results.put(self._finish(prev, dim))
                prev = (b, n, done, h)
                ph["wait"] += clock() - t3
                ph["read"] += t2 - t1
                ph["launch"] += t3 - t2
            if prev is not None:
                results.put(self._finish(prev, dim))
        except BaseException as e:   # surfaced by run() on the consuming thread
            results.put(e)
        finally:
            if fut is not None:       # a read in flight writes this lane's buffers
                try:
                    fut.result()
                except BaseException:
                    pass
            reader.shutdown(wait=True)
            with self._lock:
                for key, v in ph.items():
                    self.phase[key] += v
            results.put(None)

    @staticmethod
    def _finish(p, dim):
        b, n, done, h = p
        done.synchronize()
        return b, h[:n * dim].numpy().reshape(n, dim).copy()

    def run(self, batches):
        import queue
        results, stop = queue.Queue(), []
        lanes = [threading.Thread(target=self._lane, args=(k, batches, results, stop), daemon=True)
                 for k in range(len(self.exs))]
        for t in lanes:
            t.start()
        live, err = len(lanes), None
        try:
            while live:
                r = results.get()
                if r is None:
                    live -= 1
                elif isinstance(r, BaseException):
                    err = err or r
                    stop.append(1)
                elif err is None:
                    yield r
        finally:
            stop.append(1)
            for t in lanes:
                t.join()
            # a lane that stopped early (its own error, a peer's, or the caller
            # abandoning the generator) may have left its last batch queued: the
            # H2D from its pinned buffer, the forward and the D2H still run on
            # its stream.  Drain them before the buffers can be freed or reused
            for s in self.streams + self.copy_streams:
                s.synchronize()
        if err is not None:
            raise err


def extract_stream(table, make_runner, batch=64, ragged=False):
    """(keys, [N, dim] float32) of every utterance of `table`, in its order.
    make_runner(batches) -> an object whose run(batches) yields (batch index,
    [n, dim] embeddings) in any order.  ragged: plan_batches' ragged mode (the
    runner must take (L, items, lens) batches: LanePool)."""
    plans, batches = plan_batches(table.T, batch, table.keys, ragged=ragged)
    comb = None
    for bid, rows in make_runner(batches).run(batches):
        if comb is None:
            comb = Combiner(plans, rows.shape[1])
        comb.add_batch(batches[bid][1], rows)
    if comb is None:
        return list(table.keys), None
    assert comb.done == len(plans), (comb.done, len(plans))
    return list(table.keys), comb.out


def extract_entries(entries, extractors, batch=64, cmn=True, threads=None, ragged=None,
                    device_reader=None):
    """The GPU pipeline over scp entries [(key, rxfile)] with `extractors`
    (one lane each: same device and weights) -> (keys, [N, dim] float32).
    ragged: batch chunks of different lengths together (vox_embed_lens);
    None = wherever the model's plan supports it (Extractor.supports_lengths),
    else equal-length batches.  device_reader: decode + CMN on the GPU
    (vox_cm_chunks_device; whole "CM " matrices only); None = the host reader.
    The embeddings are the same bits either way."""
    table = ChunkTable(entries, threads)
    dim = extractors[0].dim
    if not len(table):
        return [], np.zeros((0, dim), np.float32)
    if table.feat_dim != extractors[0].feat_dim:
        raise ValueError(f"feature dim {table.feat_dim} != model {extractors[0].feat_dim}")
    if ragged is None:
        ragged = extractors[0].supports_lengths()
    return extract_stream(table, lambda batches: LanePool(extractors, table, batches, cmn,
                                                          device_reader), batch, ragged=ragged)
