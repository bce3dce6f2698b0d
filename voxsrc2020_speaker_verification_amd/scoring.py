"""Consumers of the extracted embeddings: cosine / AS-norm scoring, EER and
minDCF, and the utt -> speaker-id map.

  * snorm.py (tensorflow/snorm.py:23-131): same numpy operations in the same
    order and dtypes, so results are bit-identical to the reference on the same
    numpy/BLAS; the top-400 selection uses np.partition + a descending sort of
    the selected 400, i.e. the very array `-sort(-s)[:, :400]` the reference
    averages (same mean/std bits) without a full sort of 5994 cohort scores.
  * eer_minDCF.py (tensorflow/eer_minDCF.py:43-64): EER at argmin|FNR-FPR| over
    the ROC points of sklearn's roc_curve(drop_intermediate=True) (restated
    here, no sklearn needed), minDCF with p_target = 0.01.
  * utt2id.py (utt2id.py:20-53): speaker list order -> integer id, including
    the reference's argv pairing loop.
"""

from __future__ import annotations

import os

import numpy as np

from .kaldi import read_vec_flt_ark


# ------------------------------------------------------------------ snorm.py
def l2norm(x, axis=0, keepdims=True):
    return x / np.linalg.norm(x, axis=axis, keepdims=keepdims)


def read_xvector(ark):
    return {utt: l2norm(vec, axis=0) for utt, vec in read_vec_flt_ark(ark)}


def read_spk2utt(path):
    spk2utt = {}
    with open(path, "r") as f:
        for line in f:
            t = line.strip().split()
            spk2utt[t[0]] = t[1:]
    return spk2utt


def speaker_xvectors(xvectors, spk2utt):
    """Per-speaker mean of l2-normed utterance vectors (not re-normalised)."""
    utt_to_spk = {}
    for spk, utts in spk2utt.items():
        for utt in utts:
            utt_to_spk[utt] = spk
    groups = {}
    for utt, vec in xvectors.items():
        if utt in utt_to_spk:
            groups.setdefault(utt_to_spk[utt], []).append(vec)
    return {spk: np.mean(l2norm(np.array(v), axis=1), axis=0) for spk, v in groups.items()}


def speaker_means(keys, emb, spk2utt):
    """speaker_xvectors({k: l2norm(v) for k, v in zip(keys, emb)}, spk2utt) --
    the cohort assembly of snorm.py:45-67 on the raw embeddings -- without a
    per-utterance Python step, for VoxCeleb2-dev scale (1.09 M x 256).  Same
    result bit for bit: the same dict semantics (a repeated key keeps its first
    position and its last vector; an utterance listed under several speakers
    belongs to the last), speakers in order of their first utterance, the two
    row l2norms on the same contiguous float32 rows (a row reduction does not
    depend on the rows around it) and np.mean over each speaker's rows in
    utterance order.  Returns (speaker keys, [n_spk, D] float32)."""
    from concurrent.futures import ThreadPoolExecutor
    from itertools import repeat
    emb = np.asarray(emb)
    last = dict(zip(keys, range(len(keys))))          # {k: v} semantics
    ukeys = list(last)
    rows = np.fromiter(last.values(), dtype=np.int64, count=len(last))
    spks = list(spk2utt)
    u2s = {}
    for si, spk in enumerate(spks):
        u2s.update(dict.fromkeys(spk2utt[spk], si))   # last speaker wins
    si = np.fromiter(map(u2s.get, ukeys, repeat(-1)), dtype=np.int64, count=len(ukeys))
    keep = si >= 0
    rows, si = rows[keep], si[keep]
    if not len(rows):
        return [], np.zeros((0,) + emb.shape[1:], emb.dtype)
    uniq, first = np.unique(si, return_index=True)
    order = uniq[np.argsort(first, kind="stable")]        # speakers by first utterance
    rank_of = np.empty(len(spks), np.int64)
    rank_of[order] = np.arange(len(order))
    perm = np.argsort(rank_of[si], kind="stable")          # utterance order within a speaker
    src = rows[perm]
    counts = np.bincount(rank_of[si], minlength=len(order))
    ends = np.cumsum(counts)
    starts = ends - counts
    grouped = np.empty((len(src),) + emb.shape[1:], dtype=np.result_type(emb.dtype, np.float32))
    means = np.empty((len(order),) + emb.shape[1:], dtype=grouped.dtype)

    # numpy releases the GIL in its loops: rows (and speakers) in blocks over a
    # few threads; every row / speaker is computed by the same calls as above
    def norm_rows(lo, hi):
        grouped[lo:hi] = l2norm(l2norm(emb[src[lo:hi]], axis=1), axis=1)

    def mean_spk(lo, hi):
        for j in range(lo, hi):
            means[j] = np.mean(grouped[starts[j]:ends[j]], axis=0)

    try:
        nt = min(16, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        nt = min(16, os.cpu_count() or 1)
    with ThreadPoolExecutor(nt) as pool:
        step = max(4096, -(-len(src) // (4 * nt)))
        list(pool.map(lambda lo: norm_rows(lo, min(lo + step, len(src))), range(0, len(src), step)))
        sstep = max(64, -(-len(order) // (4 * nt)))
        list(pool.map(lambda lo: mean_spk(lo, min(lo + sstep, len(order))),
                      range(0, len(order), sstep)))
    return [spks[i] for i in order], means


def cohort_xvectors(cohort_ark, cohort_spk2utt):
    return speaker_xvectors(read_xvector(cohort_ark), read_spk2utt(cohort_spk2utt))


def projection_cohort(weight_matrix):
    """`--weight_matrix` cohort (snorm.py:77-80): rows of the l2-normed
    projection matrix; here an array, not a pickle."""
    return {i: l2norm(weight_matrix[i]) for i in range(len(weight_matrix))}


def cohort_mean_std(trial_xvectors, cohort, topk=400, block=1024):
    utt = list(trial_xvectors)
    trial = np.array(list(trial_xvectors.values()))
    cmat_t = np.transpose(np.array(list(cohort.values())))
    mean_d, std_d = {}, {}
    for i in range(0, len(trial), block):
        j = min(i + block, len(trial))
        s = np.matmul(trial[i:j, :], cmat_t)
        k = min(topk, s.shape[1])
        if k < s.shape[1]:
            part = np.partition(s, s.shape[1] - k, axis=1)[:, s.shape[1] - k:]
        else:
            part = s
        top = (-1 * np.sort(-part, axis=1))[:, :k]
        m, sd = np.mean(top, axis=1), np.std(top, axis=1)
        for r in range(i, j):
            mean_d[utt[r]], std_d[utt[r]] = m[r - i], sd[r - i]
    return mean_d, std_d


def cohort_mean_std_gpu(trial_xvectors, cohort, topk=400, device=0):
    """cohort_mean_std on the GPU (vox_asnorm_stats: fp32 MFMA score GEMM +
    exact radix top-k select, libvoxemb).  Same inputs and outputs; scores
    are summed in a different order than numpy's sgemm, so a trial whose k-th
    and (k+1)-th cohort scores tie within float rounding may pick the other
    member (the reference's own choice there is BLAS-dependent too)."""
    import ctypes as C
    import torch
    from ._native import check, lib
    utt = list(trial_xvectors)
    trial = np.ascontiguousarray(np.array(list(trial_xvectors.values())), dtype=np.float32)
    cmat = np.ascontiguousarray(np.array(list(cohort.values())), dtype=np.float32)
    dev = torch.device("cuda", device)
    # the library also selects the operands' device itself (hipPointerGetAttributes)
    with torch.cuda.device(dev):
        td, cd = torch.from_numpy(trial).to(dev), torch.from_numpy(cmat).to(dev)
        md = torch.empty(len(utt), dtype=torch.float32, device=dev)
        sd = torch.empty_like(md)
        stream = torch.cuda.current_stream(dev).cuda_stream
        check(lib().vox_asnorm_stats(C.c_void_p(td.data_ptr()), trial.shape[0],
                                     C.c_void_p(cd.data_ptr()), cmat.shape[0], trial.shape[1],
                                     int(topk), C.c_void_p(md.data_ptr()),
                                     C.c_void_p(sd.data_ptr()), C.c_void_p(stream)))
    m, s = md.cpu().numpy(), sd.cpu().numpy()
    return ({u: m[i] for i, u in enumerate(utt)}, {u: s[i] for i, u in enumerate(utt)})


def cosine_scores(trial_xvectors, trial_path):
    scores = []
    with open(trial_path, "r") as f:
        for line in f:
            u1, u2 = line.strip().split()[-2:]
            scores.append((u1, u2, np.dot(trial_xvectors[u1], trial_xvectors[u2])))
    return scores


def asnorm_scores(mean, std, scores):
    return [(u1, u2, 0.5 * ((s - mean[u1]) / std[u1] + (s - mean[u2]) / std[u2]))
            for (u1, u2, s) in scores]


def write_scores(path, scores):
    with open(path, "w") as f:
        for u1, u2, s in scores:
            print(u1, u2, s, file=f)


# ------------------------------------------------------------------ eer_minDCF.py
def roc_curve(y_true, y_score):
    """sklearn.metrics.roc_curve(y_true, y_score, pos_label=1,
    drop_intermediate=True) for binary labels {0,1}; returns fpr, tpr, thr."""
    y_true = np.asarray(y_true) == 1
    y_score = np.asarray(y_score, dtype=np.float64)
    order = np.argsort(y_score, kind="mergesort")[::-1]
    y_score = y_score[order]
    y = y_true[order].astype(np.float64)
    distinct = np.where(np.diff(y_score))[0]
    idx = np.r_[distinct, y.size - 1]
    tps = np.cumsum(y, dtype=np.float64)[idx]
    fps = 1 + idx - tps
    thr = y_score[idx]
    if len(fps) > 2:
        keep = np.where(np.r_[True, np.logical_or(np.diff(fps, 2), np.diff(tps, 2)), True])[0]
        fps, tps, thr = fps[keep], tps[keep], thr[keep]
    tps = np.r_[0, tps]
    fps = np.r_[0, fps]
    thr = np.r_[np.inf, thr]
    fpr = fps / fps[-1] if fps[-1] > 0 else np.full(fps.shape, np.nan)
    tpr = tps / tps[-1] if tps[-1] > 0 else np.full(tps.shape, np.nan)
    return fpr, tpr, thr


def compute_eer_and_min_dcf(y, y_pred, c_miss=1.0, c_fa=1.0, p_target=0.01):
    fprs, tprs, thresholds = roc_curve(y, y_pred)
    fnrs = 1.0 - tprs
    i = np.nanargmin(np.absolute(fnrs - fprs))
    eer, eer_thr = fprs[i], thresholds[i]
    c_det = c_miss * fnrs * p_target + c_fa * fprs * (1 - p_target)
    j = int(np.argmin(c_det)) if len(c_det) else 0
    min_c_det = c_det[j] if len(c_det) else float("inf")
    c_def = min(c_miss * p_target, c_fa * (1 - p_target))
    return eer, eer_thr, min_c_det / c_def, thresholds[j]


def read_trials(path):
    pair_label = {}
    with open(path) as f:
        for line in f:
            label, u1, u2 = line.strip().split()
            pair_label[(u1, u2)] = int(label)
    return pair_label


def read_scores(path):
    pair_score = {}
    with open(path) as f:
        for line in f:
            u1, u2, s = line.strip().split()
            pair_score[(u1, u2)] = float(s)
    return pair_score


def eer_from_files(trial_path, score_path, c_miss=1.0, c_fa=1.0, p_target=0.01):
    labels, scores = read_trials(trial_path), read_scores(score_path)
    y = [labels[p] for p in labels]
    s = [scores[p] for p in labels]
    return compute_eer_and_min_dcf(y, s, c_miss, c_fa, p_target)


# ------------------------------------------------------------------ utt2id.py
def read_spk(path):
    with open(path, "r") as f:
        spks = [ln.strip() for ln in f.readlines()]
    return {s: i for i, s in enumerate(spks)}


def read_utt2spk(path, spk2id):
    out = {}
    with open(path, "r") as f:
        for line in f.readlines():
            utt, spk = line.strip().split()
            if spk in spk2id:
                out[utt] = spk2id[spk]
    return out


def utt2id_main(argv):
    """utt2id.py's __main__ (:48-53): pairs argv[i], argv[i+1] for i in
    1 .. len(argv)//2 - 1 (so more than one pair misreads files, as there)."""
    assert len(argv) % 2 == 0
    out = {}
    for i in range(1, len(argv) // 2):
        out.update(read_utt2spk(argv[i], read_spk(argv[i + 1])))
    return out
