"""The N>1 extraction path on CPU: 2 ranks over gloo, split_scp shards,
variable-size all-gather, merged ark == `cat` of the per-rank arks
(eval_inference_model.sh:38-39), cohort speaker means on rank 0."""

import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_embed(x):
    # deterministic per-utterance "embedding": depends only on that utterance
    return np.concatenate([x.mean(1), x.std(1)], axis=1).astype(np.float32)[:, :8]


def _items(n_utts):
    rng = np.random.default_rng(0)
    lens = rng.integers(25, 1300, size=n_utts)
    feats = [(f"spk{i % 3}-u{i:03d}", rng.standard_normal((int(L), 4)).astype(np.float32))
             for i, L in enumerate(lens)]

    def items(rank, world):
        from voxsrc2020_speaker_verification_amd.partition import shard
        return shard(feats, rank, world)
    return feats, items


def _worker(rank, world, port, outdir, n_utts, streamed=False, all_gather=False):
    import torch.distributed as dist
    from voxsrc2020_speaker_verification_amd import dp_extract
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    _, items = _items(n_utts)
    spk2utt = os.path.join(outdir, "spk2utt")
    shard_fn = None
    if streamed:   # the CLI's form: the rank's scp lines streamed (stream.py), never decoded whole
        from voxsrc2020_speaker_verification_amd import kaldi, stream
        from voxsrc2020_speaker_verification_amd.partition import shard

        def shard_fn(r, w):
            table = stream.ChunkTable(shard(kaldi.read_scp(os.path.join(outdir, "feats.scp")), r, w), 2)
            return stream.extract_stream(
                table, lambda b: stream.SyncRunner(table, _fake_embed, cmn=False), 3)
    keys, emb = dp_extract.run(rank, world, items, _fake_embed, 8, os.path.join(outdir, "xvector"),
                               batch=3, cohort_spk2utt=spk2utt, extract_shard=shard_fn,
                               all_gather=all_gather)
    # rank 0 receives everything; the others only with all_gather
    got = len(keys) if emb is None else emb.shape[0]
    with open(os.path.join(outdir, f"recv{rank}"), "w") as f:
        f.write(f"{len(keys)} {got}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_utts,streamed,all_gather",
                         [(2, 11, False, False), (3, 7, False, True), (3, 7, False, False),
                          (2, 11, True, False)])
def test_dp_extract_gloo(tmp_path, world, n_utts, streamed, all_gather):
    import torch.multiprocessing as mp
    from voxsrc2020_speaker_verification_amd import kaldi
    from voxsrc2020_speaker_verification_amd.extract import embed_utterances
    feats, _ = _items(n_utts)
    with open(tmp_path / "spk2utt", "w") as f:
        for s in range(3):
            f.write(f"spk{s} " + " ".join(k for k, _ in feats if k.startswith(f"spk{s}-")) + "\n")
    if streamed:
        with open(tmp_path / "feats.ark", "wb") as fa, open(tmp_path / "feats.scp", "w") as fs:
            for k, m in feats:
                rec, off = kaldi.format_mat_flt(k, m)
                fs.write(f"{k} {tmp_path / 'feats.ark'}:{fa.tell() + off}\n")
                fa.write(rec)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_utts, streamed, all_gather),
             nprocs=world, join=True)
    recv = [open(tmp_path / f"recv{r}").read() for r in range(world)]
    full = f"{n_utts} {n_utts}"
    assert recv == [full] * world if all_gather else recv == [full] + ["0 0"] * (world - 1)
    # merged ark is byte-identical to the concatenation of the per-rank arks
    cat = b"".join(open(tmp_path / f"xvector.{r + 1}.ark", "rb").read() for r in range(world))
    assert open(tmp_path / "xvector.ark", "rb").read() == cat
    got = dict(kaldi.read_vec_flt_ark(str(tmp_path / "xvector.ark")))
    assert list(got) == [k for k, _ in feats]
    exp = embed_utterances(feats, _fake_embed, 8, batch=5)
    for (k, _), e in zip(feats, exp):
        np.testing.assert_array_equal(got[k], e)
    coh = np.load(tmp_path / "xvector.cohort.npy")
    assert coh.shape == (3, 8)
    # the vectorised cohort == snorm.py's per-utterance dict path, bit for bit
    from voxsrc2020_speaker_verification_amd import scoring
    spk = scoring.speaker_xvectors({k: scoring.l2norm(v, axis=0) for k, v in got.items()},
                                   scoring.read_spk2utt(str(tmp_path / "spk2utt")))
    assert np.array_equal(coh, np.array(list(spk.values()), np.float32))
    assert open(tmp_path / "xvector.cohort.keys").read().split() == list(spk)


def _failing_worker(rank, world, port, outdir):
    import torch.distributed as dist
    from voxsrc2020_speaker_verification_amd import dp_extract
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(rank)
    # rank 1 holds a 10-frame utterance: the chunk rule divides by zero there
    L = 10 if rank == 1 else 40
    feats = [(f"u{rank}", rng.standard_normal((L, 4)).astype(np.float32))]
    try:
        dp_extract.run(rank, world, lambda r, w: feats, _fake_embed, 8, None, batch=3)
        res = "ok"
    except ZeroDivisionError:
        res = "own"
    except RuntimeError as e:
        res = "peer" if "rank(s) [1]" in str(e) else repr(e)
    with open(os.path.join(outdir, f"r{rank}"), "w") as f:
        f.write(res)
    dist.destroy_process_group()


def test_dp_extract_rank_failure_aborts_all(tmp_path):
    """A failing shard makes every rank abort before the gathers (no hang)."""
    import torch.multiprocessing as mp
    world = 3
    mp.spawn(_failing_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = [open(tmp_path / f"r{r}").read() for r in range(world)]
    assert got == ["peer", "own", "peer"]


def _resume_worker(rank, world, port, outdir, n_utts):
    import torch.distributed as dist
    from voxsrc2020_speaker_verification_amd import dp_extract
    from voxsrc2020_speaker_verification_amd.partition import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    feats, items = _items(n_utts)

    def counted(x):   # marks that this rank ran the extractor
        with open(os.path.join(outdir, f"ran{rank}"), "a") as f:
            f.write("x")
        return _fake_embed(x)
    dp_extract.run(rank, world, items, counted, 8, os.path.join(outdir, "xvector"), batch=3,
                   resume=True, shard_keys=lambda r, w: [k for k, _ in shard(feats, r, w)])
    dist.barrier()
    dist.destroy_process_group()


def test_dp_extract_resume_skips_finished_shards(tmp_path):
    """SURVEY §5 resume: a second run with resume=True reuses the ranks whose
    xvector.<i>.ark/.scp hold their whole shard and recomputes the others (here
    rank 2's ark was cut short, as by a crash); the merged output is identical."""
    import torch.multiprocessing as mp
    world, n = 3, 10
    mp.spawn(_resume_worker, args=(world, _free_port(), str(tmp_path), n), nprocs=world, join=True)
    first = open(tmp_path / "xvector.ark", "rb").read()
    assert sorted(p.name for p in tmp_path.glob("ran*")) == ["ran0", "ran1", "ran2"]
    for p in tmp_path.glob("ran*"):
        p.unlink()
    ark2 = tmp_path / "xvector.3.ark"
    ark2.write_bytes(ark2.read_bytes()[:-7])     # truncated record
    (tmp_path / "xvector.ark").unlink()
    mp.spawn(_resume_worker, args=(world, _free_port(), str(tmp_path), n), nprocs=world, join=True)
    assert sorted(p.name for p in tmp_path.glob("ran*")) == ["ran2"]
    assert open(tmp_path / "xvector.ark", "rb").read() == first
    assert not list(tmp_path.glob("*.part*"))


def test_atomic_writer_failure_publishes_nothing(tmp_path):
    """A write that raises leaves neither the ark/scp pair nor .part files."""
    from voxsrc2020_speaker_verification_amd.kaldi import VectorWriter
    base = str(tmp_path / "xvector.1")
    with pytest.raises(RuntimeError):
        with VectorWriter(base, atomic=True) as w:
            w.write("a", np.ones(4, np.float32))
            raise RuntimeError("extractor died")
    assert not list(tmp_path.iterdir())


def test_resume_requires_matching_run_tag(tmp_path):
    """--resume reuses a per-rank pair only if it was made with the same weights
    and precision (the tag file beside it); otherwise the shard is recomputed."""
    from voxsrc2020_speaker_verification_amd import dp_extract
    from voxsrc2020_speaker_verification_amd.extract import write_vectors
    blob = tmp_path / "m.blob"
    blob.write_bytes(b"weights-1")
    keys = ["u1", "u2"]
    emb = np.arange(8, dtype=np.float32).reshape(2, 4)
    base = str(tmp_path / "xvector")
    write_vectors(base + ".1", keys, emb, atomic=True)
    tag = dp_extract.run_tag(str(blob), "bf16")
    assert dp_extract.completed_shard(base, 0, keys, 4, tag) is None      # no tag file yet
    dp_extract._write_tag(base + ".1", tag)
    assert np.array_equal(dp_extract.completed_shard(base, 0, keys, 4, tag), emb)
    assert dp_extract.completed_shard(base, 0, keys, 4, dp_extract.run_tag(str(blob), "fp32")) is None
    blob.write_bytes(b"weights-2")
    assert dp_extract.completed_shard(base, 0, keys, 4, dp_extract.run_tag(str(blob), "bf16")) is None
