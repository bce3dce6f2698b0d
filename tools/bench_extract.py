"""The product extraction path on real-length inputs (tf_extract.py:85-113;
SURVEY §5 "long-context / sequence scaling"): seeded synthetic utterances with
VoxCeleb-like lengths (uniform 200-2,000 frames) in a Kaldi compressed (CM)
feature ark + scp, as `copy-feats --compress=true` writes them
(prepare_data.sh:69), extracted through stream.extract_entries (the
extract.py / dp_extract.py pipeline: header planning, native batched reader,
lanes) in a fresh child process that reports its own peak RSS.

Reports utt/s and frames/s of the whole path (planning + decode + CMN + H2D +
forward + D2H + combination; writing the ark timed separately), the plan-build
count, peak RSS for N and 2N utterances, and the fixed-shape frames/s of the
bench workload (B=256, T=200) on the same device for comparison.

    python tools/bench_extract.py [--utts 4096] [--lanes 4] [--out profiles/r05_extract.json]
"""
import argparse
import json
import os
import resource
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_ark(base, n, feat_dim, seed, lo=200, hi=2000):
    """n utterances, lengths uniform in [lo, hi] frames, CM-compressed on the
    device (vox_cm_compress_device), written as <base>.ark / <base>.scp."""
    import numpy as np
    import torch
    from voxsrc2020_speaker_verification_amd.frontend import cm_compress_device, format_cm_record
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n)
    dev = torch.device("cuda", 0)
    with open(base + ".ark", "wb") as fa, open(base + ".scp", "w") as fs:
        for b0 in range(0, n, 256):
            part = lens[b0:b0 + 256]
            fo = np.zeros(len(part) + 1, np.int64)
            fo[1:] = np.cumsum(part)
            feats = torch.randn(int(fo[-1]), feat_dim, device=dev) * 3 + 1
            _, blob, boff = cm_compress_device(feats, fo, decode=False)
            hb = blob.cpu().numpy()
            for i, T in enumerate(part):
                key = f"spk{(b0 + i) % 97:03d}-utt{b0 + i:06d}"
                rec, off = format_cm_record(key, hb[boff[i]:boff[i + 1]], int(T))
                pos = fa.tell()
                fa.write(rec)
                fs.write(f"{key} {base}.ark:{pos + off}\n")
    return int(lens.sum())


def child(args):
    """One extraction run in this process; prints a JSON line."""
    import numpy as np
    import torch
    from bench import weights_blob
    from voxsrc2020_speaker_verification_amd import extract, kaldi, stream
    torch.cuda.set_device(0)
    blob = weights_blob(args.model, 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    lanes = [__import__("voxsrc2020_speaker_verification_amd.extractor", fromlist=["Extractor"])
             .Extractor(blob, device=0, precision="bf16") for _ in range(args.lanes)]
    entries = kaldi.read_scp(args.scp)
    torch.cuda.synchronize()
    ragged = {"ragged": True, "exact": False, "auto": None}[args.mode]
    if ragged is None:
        ragged = lanes[0].supports_lengths()
    st0 = [ex.plan_stats() for ex in lanes]
    t0 = time.perf_counter()
    table = stream.ChunkTable(entries, args.threads)
    plans, batches = stream.plan_batches(table.T, args.batch, table.keys, ragged=ragged)
    t_plan = time.perf_counter() - t0
    pools = []

    devread = {"auto": None, "host": False, "device": True}[args.reader]

    def make_pool(b):
        pools.append(stream.LanePool(lanes, table, b, device_reader=devread))
        return pools[-1]

    keys, emb = stream.extract_stream(table, make_pool, args.batch, ragged=ragged)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    el = t1 - t0
    # the same pass again with every plan resident (a long job's steady state)
    keys2, emb2 = stream.extract_stream(table, make_pool, args.batch, ragged=ragged)
    torch.cuda.synchronize()
    t_warm = time.perf_counter() - t1
    assert keys2 == keys and np.array_equal(emb2.view(np.uint32), emb.view(np.uint32))
    t1 = time.perf_counter()
    extract.write_vectors(args.wspec, keys, emb)
    t_write = time.perf_counter() - t1
    frames = int(table.T.sum())
    st = [{k: v - s0[k] for k, v in s1.items()} for s0, s1 in zip(st0, (ex.plan_stats() for ex in lanes))]
    pad = sum(b[0] * len(b[1]) for b in batches)
    for ex in lanes:
        ex.close()
    print(json.dumps({
        "utts": len(keys), "frames": frames, "chunks": sum(len(p) for p in plans),
        "batches": len(batches), "distinct_lengths": len({b[0] for b in batches}),
        "mode": "ragged" if ragged else "exact", "padded_frames_frac": round(frames_chunks(plans) / pad, 4),
        "seconds": round(el, 4), "plan_s": round(t_plan, 4), "write_s": round(t_write, 4),
        "utt_per_s": round(len(keys) / el, 1), "frames_per_s": round(frames / el, 1),
        "warm_seconds": round(t_warm, 4), "warm_frames_per_s": round(frames / t_warm, 1),
        "reader": "device" if pools[0].devread else "host",
        "lane_phase_s": {k: round(v, 4) for k, v in pools[0].phase.items()},
        "warm_lane_phase_s": {k: round(v, 4) for k, v in pools[1].phase.items()},
        "plans_built": sum(s["built"] for s in st), "plan_hits": sum(s["hits"] for s in st),
        "plans_dropped": sum(s["dropped"] for s in st), "lanes": args.lanes,
        "batch": args.batch, "reader_threads": table.threads,
        "peak_rss_mb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024, 1)}))


def frames_chunks(plans):
    return sum(L for p in plans for _, L in p)


def fixed_shape_fps(model, B=256, T=200, steps=10):
    import torch
    from bench import bench_features, weights_blob
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    torch.cuda.set_device(0)
    blob = weights_blob(model, 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    with Extractor(blob, device=0, precision="bf16") as ex:
        x = torch.from_numpy(bench_features(B, T, 80)).cuda()
        out = torch.empty((B, ex.dim), device=x.device)
        s = torch.cuda.Stream()
        for _ in range(3):
            ex.run_device(x, out, s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            ex.run_device(x, out, s)
        torch.cuda.synchronize()
        return B * T * steps / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=4096)
    ap.add_argument("--lanes", default="4", help="comma list: one run per lane count")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--model", default="res2net50_w24_s4_c32")
    ap.add_argument("--dir", default="/tmp/voxemb_bench_extract")
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--scp", default=None)
    ap.add_argument("--wspec", default=None)
    ap.add_argument("--reader", default="auto", choices=["auto", "host", "device"],
                    help="decode + CMN on the host threads or on the GPU (vox_cm_chunks_device)")
    ap.add_argument("--mode", default="auto", choices=["auto", "ragged", "exact"],
                    help="ragged batches (vox_embed_lens) or equal-length batches")
    args = ap.parse_args()
    if args.child:
        args.lanes = int(args.lanes)
        return child(args)

    os.makedirs(args.dir, exist_ok=True)
    res = {"model": args.model, "lengths": "uniform 200-2000 frames (seeded)", "format": "CM ark"}
    res["fixed_shape_frames_per_s"] = round(fixed_shape_fps(args.model), 1)
    runs = []
    for n in (args.utts, 2 * args.utts):
        base = os.path.join(args.dir, f"feats{n}")
        if not os.path.exists(base + ".scp"):
            t0 = time.perf_counter()
            make_ark(base, n, 80, seed=n)
            print(f"wrote {n} utterances in {time.perf_counter() - t0:.1f} s", file=sys.stderr)
        for lanes in [int(s) for s in args.lanes.split(",")]:
            if n != args.utts and lanes != int(args.lanes.split(",")[-1]):
                continue   # the doubled set: RSS check at the last lane count only
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--scp", base + ".scp",
                   "--wspec", os.path.join(args.dir, f"xv{n}_{lanes}"), "--lanes", str(lanes),
                   "--batch", str(args.batch), "--model", args.model, "--mode", args.mode,
                   "--reader", args.reader]
            if args.threads:
                cmd += ["--threads", str(args.threads)]
            r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
            if r.returncode != 0:
                print(r.stderr[-3000:], file=sys.stderr)
                raise SystemExit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d["frac_of_fixed_shape"] = round(d["frames_per_s"] / res["fixed_shape_frames_per_s"], 4)
            print(json.dumps(d), flush=True)
            runs.append(d)
    res["runs"] = runs
    a = [d for d in runs if d["utts"] == args.utts]
    b = [d for d in runs if d["utts"] == 2 * args.utts]
    if a and b:
        res["peak_rss_mb"] = {str(args.utts): a[-1]["peak_rss_mb"], str(2 * args.utts): b[-1]["peak_rss_mb"]}
    print(json.dumps(res))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
