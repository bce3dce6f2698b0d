"""Host chunk reader alone (vox_read_chunks_ragged: read + Kaldi CM decode +
sliding CMN, tf_extract.py:63 / :85-90), no GPU forward: frames/s over
one pass of a synthetic CM scp in ragged batches of 64, per library and thread
count.  LIBS="name ..." picks voxsrc2020_speaker_verification_amd/libvoxemb_<name>.so
("cur" = libvoxemb.so) for an A/B; each (lib, threads) runs in its own child.

  python3 tools/bench_reader.py --utts 2048 --threads 1,4,8,16 --out r.json
"""

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(scp, threads, reps):
    import numpy as np
    from voxsrc2020_speaker_verification_amd import kaldi, stream
    table = stream.ChunkTable(kaldi.read_scp(scp), threads=threads)
    _, batches = stream.plan_batches(table.T, 64, ragged=True)
    frames = sum(sum(b[2]) for b in batches)
    buf = np.zeros(64 * stream.MAX_FRAMES * table.feat_dim, np.float32)
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        for Lp, items, lens in batches:
            table.read_ragged(items, lens, Lp, buf)
        best = max(best, frames / (time.perf_counter() - t0))
    print(json.dumps({"threads": threads, "frames": frames, "frames_per_s": best}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, default=2048)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp/voxemb_bench_reader")
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", nargs=2, metavar=("SCP", "THREADS"))
    args = ap.parse_args()
    if args.child:
        return child(args.child[0], int(args.child[1]), args.reps)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from bench_extract import make_ark
    os.makedirs(args.dir, exist_ok=True)
    base = os.path.join(args.dir, f"cm{args.utts}")
    if not os.path.exists(base + ".scp"):
        make_ark(base, args.utts, 80, seed=7)
    pkg = os.path.join(ROOT, "voxsrc2020_speaker_verification_amd")
    runs = []
    for name in os.environ.get("LIBS", "cur").split():
        lib = os.path.join(pkg, "libvoxemb.so" if name == "cur" else f"libvoxemb_{name}.so")
        for th in [int(t) for t in args.threads.split(",")]:
            env = dict(os.environ, VOXEMB_LIB=lib)
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--reps", str(args.reps),
                                "--child", base + ".scp", str(th)], env=env, capture_output=True,
                               text=True, cwd=ROOT, timeout=600)
            if r.returncode:
                sys.stderr.write(r.stderr[-3000:])
                raise SystemExit(r.returncode)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d["lib"] = name
            runs.append(d)
            print(name, th, f"{d['frames_per_s'] / 1e6:.2f} M frames/s", flush=True)
    res = {"what": "host reader alone: read + CM decode + sliding CMN, ragged batches of 64",
           "utts": args.utts, "runs": runs}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
