"""Streaming extraction of a Kaldi feature scp with bounded host memory.

The reference (tensorflow/tf_extract.py:85-113) streams: a reader process
decodes one utterance at a time through the `apply-cmvn-sliding` pipe (:63)
into a Queue(32), and the session runs each <= 1000-frame chunk on its own
(:96-108).  Here the same results come out of three stages that overlap:

  1. planning (headers only): every utterance's frame count from its matrix
     header (`vox_mat_shapes`), the chunk rule (:96-107) applied, and the chunks
     bucketed by length over the whole shard -- equal-length chunks batch
     together bit for bit (embeddings are batch-independent), and the shard is
     one planning window, so real length distributions still give full batches;
  2. reading: each batch's chunks decoded, CMN'd and sliced straight into a
     pinned host buffer by the native reader (`vox_read_chunks`, host threads),
     one batch ahead of the GPU, into a bounded ring of buffers;
  3. compute: the batches go round-robin to `lanes` extraction handles, each
     with its own stream, device buffers and resident plans; the H2D copy, the
     forward and the D2H copy of one batch are queued on its lane's stream.

Host memory is the ring (a few batches of features) plus one embedding per
utterance; nothing grows with the features of the shard.  The per-utterance
combination (length-weighted mean, :108-111) is the float32 arithmetic of
`extract.embed_utterances`, so the arks are byte-identical to it.
"""

from __future__ import annotations

import collections
import ctypes as C
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ._native import check, lib
from .extractor import MIN_FRAMES, chunk_plan
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

    def __len__(self):
        return len(self.keys)

    def read(self, items, L, out, cmn=True):
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
                                    CMN_WINDOW if cmn else 0, C.c_void_p(ptr), self.threads))


def plan_batches(lengths, batch, keys=None):
    """The chunk rule over every utterance, equal-length chunks bucketed:
    -> (per-utterance chunk plans, [(L, [(u, ci, start), ...]), ...]).  Buckets
    keep scp order inside; batches are ordered by size (frames) descending, so
    the first batch sizes the device workspace once.  An utterance shorter than
    25 frames raises ZeroDivisionError, as tf_extract.py:111 does."""
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
    batches = [(L, items[b:b + batch]) for L, items in buckets.items()
               for b in range(0, len(items), batch)]
    batches.sort(key=lambda b: -b[0] * len(b[1]))
    return plans, batches


class Combiner:
    """Per-utterance length-weighted mean of its chunk embeddings in chunk
    order (extract.embed_utterances' float32 arithmetic, tf_extract.py:108-111);
    multi-chunk utterances wait here until their last chunk arrives."""

    def __init__(self, plans, dim):
        self.plans = plans
        self.out = np.empty((len(plans), dim), np.float32)
        self._part = {}
        self.done = 0

    def add(self, u, ci, row):
        plan = self.plans[u]
        if len(plan) == 1:
            rows = [row]
        else:
            got = self._part.setdefault(u, {})
            got[ci] = row
            if len(got) < len(plan):
                return
            rows = [got[i] for i in range(len(plan))]
            del self._part[u]
        acc = 0
        for r, (_, L) in zip(rows, plan):
            acc = acc + r * L
        self.out[u] = acc / sum(L for _, L in plan)
        self.done += 1


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
    """`lanes` extraction handles on one device, each with its own stream,
    input / output device buffers sized for the largest batch, and resident
    plans; a ring of pinned host buffers filled by the native reader one or
    more batches ahead."""

    def __init__(self, extractors, table, batches, cmn=True, ring=None, max_pending=None):
        import torch
        self.torch = torch
        self.exs = list(extractors)
        self.table, self.cmn = table, cmn
        self.dev = torch.device("cuda", self.exs[0].device)
        F = table.feat_dim
        self.max_el = max((len(it) * L * F for L, it in batches), default=1)
        self.max_n = max((len(it) for _, it in batches), default=1)
        K = len(self.exs)
        self.ring = ring or max(3, K + 2)
        self.max_pending = max_pending or 2 * K + 2
        dim = self.exs[0].dim
        self.streams = [torch.cuda.Stream(self.dev) for _ in range(K)]
        self.d_in = [torch.empty(self.max_el, dtype=torch.float32, device=self.dev) for _ in range(K)]
        self.d_out = [torch.empty(self.max_n * dim, dtype=torch.float32, device=self.dev)
                      for _ in range(K)]
        self.h_in = [torch.empty(self.max_el, dtype=torch.float32).pin_memory() for _ in range(self.ring)]
        self.h_free = [None] * self.ring          # event after the H2D that last read h_in[k]
        self.h_out = [torch.empty(self.max_n * dim, dtype=torch.float32).pin_memory()
                      for _ in range(self.max_pending + 1)]

    def run(self, batches):
        torch = self.torch
        K, F, dim = len(self.exs), self.table.feat_dim, self.exs[0].dim
        pending = collections.deque()      # (bid, n, done event, h_out index)
        reader = ThreadPoolExecutor(max_workers=1)
        futs = {}

        def submit(b):
            k = b % self.ring
            if self.h_free[k] is not None:
                self.h_free[k].synchronize()
            L, items = batches[b]
            futs[b] = reader.submit(self.table.read, items, L, self.h_in[k], self.cmn)

        try:
            for b in range(min(self.ring - 1, len(batches))):
                submit(b)
            out_slot = 0
            for b, (L, items) in enumerate(batches):
                futs.pop(b).result()
                if b + self.ring - 1 < len(batches):
                    submit(b + self.ring - 1)
                n, k, lane = len(items), b % self.ring, b % K
                s = self.streams[lane]
                ne = n * L * F
                x = self.d_in[lane][:ne]
                o = self.d_out[lane][:n * dim]
                with torch.cuda.stream(s):
                    x.copy_(self.h_in[k][:ne], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(s)
                    self.h_free[k] = ev
                self.exs[lane].run_device(x.view(n, L, F), o.view(n, dim), s)
                while len(pending) >= self.max_pending:
                    yield self._finish(pending.popleft())
                h = self.h_out[out_slot]
                out_slot = (out_slot + 1) % len(self.h_out)
                with torch.cuda.stream(s):
                    h[:n * dim].copy_(o, non_blocking=True)
                    done = torch.cuda.Event()
                    done.record(s)
                pending.append((b, n, done, h))
                while pending and pending[0][2].query():
                    yield self._finish(pending.popleft())
            while pending:
                yield self._finish(pending.popleft())
        finally:
            reader.shutdown(wait=True)

    def _finish(self, p):
        b, n, done, h = p
        done.synchronize()
        dim = self.exs[0].dim
        return b, h[:n * dim].numpy().reshape(n, dim).copy()


def extract_stream(table, make_runner, batch=64):
    """(keys, [N, dim] float32) of every utterance of `table`, in its order.
    make_runner(batches) -> an object whose run(batches) yields (batch index,
    [n, dim] embeddings) in any order."""
    plans, batches = plan_batches(table.T, batch, table.keys)
    comb = None
    for bid, rows in make_runner(batches).run(batches):
        if comb is None:
            comb = Combiner(plans, rows.shape[1])
        for (u, ci, _), row in zip(batches[bid][1], rows):
            comb.add(u, ci, row)
    if comb is None:
        return list(table.keys), None
    assert comb.done == len(plans), (comb.done, len(plans))
    return list(table.keys), comb.out


def extract_entries(entries, extractors, batch=64, cmn=True, threads=None):
    """The GPU pipeline over scp entries [(key, rxfile)] with `extractors`
    (one lane each: same device and weights) -> (keys, [N, dim] float32)."""
    table = ChunkTable(entries, threads)
    dim = extractors[0].dim
    if not len(table):
        return [], np.zeros((0, dim), np.float32)
    if table.feat_dim != extractors[0].feat_dim:
        raise ValueError(f"feature dim {table.feat_dim} != model {extractors[0].feat_dim}")
    return extract_stream(table, lambda batches: LanePool(extractors, table, batches, cmn), batch)
