"""Cohort assembly at VoxCeleb2-dev scale (snorm.py:45-67 fed by
eval_inference_model.sh:38-51): the rank-0 tail of dp_extract.run on
synthetic embeddings -- gather of every rank's [n_r, 256] matrix to rank 0,
the merged xvector ark/scp, and the 5,994 speaker means -- timed per phase,
with the process's peak RSS after each.

    python tools/bench_cohort.py [--utts 1092009] [--speakers 5994] [--old]
    torchrun --nproc-per-node N tools/bench_cohort.py ...   (RCCL when a GPU is visible)

--old also times snorm.py's per-utterance path (scoring.speaker_xvectors on a
{key: l2norm(vec)} dict, what dp_extract ran before) and checks the two
cohort matrices are bit-identical.  Prints one JSON line (rank 0)."""

from __future__ import annotations

import argparse
import json
import os
import resource
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rss_mb():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


def synth(n_utts, n_spk, dim, rank, world, seed=7):
    """Rank `rank`'s contiguous shard of n_utts synthetic VoxCeleb2-style keys
    (id<spk>-<video>-<utt>, speakers of unequal size, in spk2utt order like a
    sorted scp) and the full spk2utt."""
    rng = np.random.default_rng(seed)
    w = rng.gamma(4.0, 1.0, n_spk)
    per = np.maximum(1, np.floor(w / w.sum() * n_utts)).astype(np.int64)
    per[: n_utts - per.sum()] += 1 if n_utts > per.sum() else 0
    while per.sum() > n_utts:
        per[np.argmax(per)] -= 1
    spk = [f"id{s:05d}" for s in range(n_spk)]
    keys = [f"{spk[s]}-v{j // 8:04d}-{j % 8:05d}" for s in range(n_spk) for j in range(per[s])]
    spk2utt, o = {}, 0
    for s in range(n_spk):
        spk2utt[spk[s]] = keys[o:o + per[s]]
        o += per[s]
    lo, hi = (len(keys) * rank) // world, (len(keys) * (rank + 1)) // world
    emb = np.random.default_rng(seed + 1 + rank).standard_normal((hi - lo, dim)).astype(np.float32)
    return keys[lo:hi], emb, spk2utt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=1092009)     # VoxCeleb2 dev
    ap.add_argument("--speakers", type=int, default=5994)
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--old", action="store_true")
    ap.add_argument("--no-write", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch
    import torch.distributed as dist
    from voxsrc2020_speaker_verification_amd import dp_extract, scoring
    from voxsrc2020_speaker_verification_amd.extract import write_vectors

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
        dev = torch.device("cuda", local)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cpu")
    t = {}
    t0 = time.perf_counter()
    keys, emb, spk2utt = synth(a.utts, a.speakers, a.dim, rank, world)
    t["synth_s"] = time.perf_counter() - t0
    rss = {"after_synth": rss_mb()}
    dist.barrier()
    t0 = time.perf_counter()
    all_keys, all_emb = dp_extract.gather_embeddings(keys, emb, device=dev, dst=0)
    t["gather_s"] = time.perf_counter() - t0
    rss["after_gather"] = rss_mb()
    line = None
    if rank == 0:
        tmp = tempfile.mkdtemp(prefix="cohort_", dir=a.out)
        try:
            if not a.no_write:
                t0 = time.perf_counter()
                write_vectors(os.path.join(tmp, "xvector"), all_keys, all_emb)
                t["merged_ark_s"] = time.perf_counter() - t0
                t["merged_ark_bytes"] = os.path.getsize(os.path.join(tmp, "xvector.ark"))
                rss["after_write"] = rss_mb()
            t0 = time.perf_counter()
            spk, cohort = scoring.speaker_means(all_keys, all_emb, spk2utt)
            t["cohort_s"] = time.perf_counter() - t0
            rss["after_cohort"] = rss_mb()
            same = None
            if a.old:
                t0 = time.perf_counter()
                xv = {k: scoring.l2norm(v, axis=0) for k, v in zip(all_keys, all_emb)}
                ref = scoring.speaker_xvectors(xv, spk2utt)
                t["cohort_old_s"] = time.perf_counter() - t0
                rss["after_old"] = rss_mb()
                same = (list(ref) == spk and np.array_equal(
                    np.array(list(ref.values()), np.float32).view(np.uint32),
                    cohort.view(np.uint32)))
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        line = {"what": "cohort assembly (dp_extract rank-0 tail)", "world": world,
                "backend": "nccl" if gpu else "gloo", "utterances": len(all_keys),
                "speakers": len(spk), "dim": a.dim,
                "cohort_shape": list(cohort.shape),
                "times": {k: (round(v, 3) if k.endswith("_s") else v) for k, v in t.items()},
                "assembly_s": round(t["gather_s"] + t["cohort_s"], 3),
                "peak_rss_mb": {k: round(v, 1) for k, v in rss.items()},
                "old_path_bit_identical": same,
                "host_cpus": os.cpu_count()}
        print(json.dumps(line))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
