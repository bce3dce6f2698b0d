"""Forward time of the headline network at small batches and long chunks: the
shapes real extraction produces (one bucket per chunk length, tf_extract.py:96-111).

For each (n, T): frames/s of graph replays of one plan, of a first (eager) call
on a fresh shape, and of k concurrent lanes (own Extractor + stream each).

    python tools/shape_sweep.py [--ns 1,2,4,8,16,32,64] [--ts 200,600,1000] [--lanes 1,2,4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8,16,32,64")
    ap.add_argument("--ts", default="200,600,1000")
    ap.add_argument("--lanes", default="1,4")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--model", default="res2net50_w24_s4_c32")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch
    from bench import weights_blob
    from voxsrc2020_speaker_verification_amd import synth
    from voxsrc2020_speaker_verification_amd.extractor import Extractor

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    blob = weights_blob(args.model, 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    lanes = [int(s) for s in args.lanes.split(",")]
    K = max(lanes)
    exs = [Extractor(blob, device=0, precision="bf16") for _ in range(K)]
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    rows = []
    for T in [int(s) for s in args.ts.split(",")]:
        for n in [int(s) for s in args.ns.split(",")]:
            x = torch.from_numpy(synth.make_features(n, T, 80, seed=5)).to(dev)
            outs = [torch.empty((n, exs[0].dim), dtype=torch.float32, device=dev) for _ in range(K)]
            torch.cuda.synchronize(dev)
            # first call on a fresh shape (plan + eager or capture)
            t0 = time.perf_counter()
            exs[0].run_device(x, outs[0], streams[0])
            torch.cuda.synchronize(dev)
            first = time.perf_counter() - t0
            r = {"n": n, "T": T, "first_ms": round(first * 1e3, 3)}
            for k in lanes:
                for i in range(k):
                    exs[i].run_device(x, outs[i], streams[i])
                    exs[i].run_device(x, outs[i], streams[i])
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    for i in range(k):
                        exs[i].run_device(x, outs[i], streams[i])
                torch.cuda.synchronize(dev)
                el = time.perf_counter() - t0
                r[f"lanes{k}_ms_per_batch"] = round(el * 1e3 / (args.steps * k), 4)
                r[f"lanes{k}_frames_per_s"] = round(args.steps * k * n * T / el, 1)
            print(json.dumps(r), flush=True)
            rows.append(r)
    for e in exs:
        e.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
