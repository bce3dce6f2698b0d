"""Does running the batch as independent sub-batches on concurrent streams fill
the kernel tails?  Times the headline workload (res2net50_w24_s4_c32, 80x200,
bf16) as one B-utterance forward on one stream vs k forwards of B/k utterances,
each on its own Extractor (own slots) and its own stream, launched round-robin.
Embeddings are batch-size independent bitwise (test_batch_256_plan_bitwise), so
the split changes no output bit; this only measures time.

    python tools/stream_overlap.py [--batch 256] [--steps 20] [--splits 1,2,4]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--model", default="res2net50_w24_s4_c32")
    args = ap.parse_args()

    import torch
    from bench import weights_blob, bench_features
    from voxsrc2020_speaker_verification_amd.extractor import Extractor

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    blob = weights_blob(args.model, 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    B = args.batch
    x = torch.from_numpy(bench_features(B, 200, 80, 0)).to(dev)
    res = {}
    ref = None
    for k in [int(s) for s in args.splits.split(",")]:
        assert B % k == 0
        b = B // k
        exs = [Extractor(blob, device=0, precision="bf16") for _ in range(k)]
        xs = [x[i * b:(i + 1) * b].contiguous() for i in range(k)]
        outs = [torch.empty((b, exs[0].dim), dtype=torch.float32, device=dev) for _ in range(k)]
        streams = [torch.cuda.Stream(dev) for _ in range(k)]
        torch.cuda.synchronize(dev)

        def step():
            for e, xi, oi, s in zip(exs, xs, outs, streams):
                e.run_device(xi, oi, s)

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        emb = torch.cat(outs).cpu()
        if ref is None:
            ref = emb
        res[k] = dict(utt_per_s=round(B * args.steps / el, 1),
                      ms_per_step=round(el * 1e3 / args.steps, 3),
                      bitwise_vs_first=bool(torch.equal(emb, ref)))
        print(f"splits={k}: {res[k]}", flush=True)
        del exs, outs
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
    print(json.dumps(dict(batch=B, steps=args.steps, results=res)))


if __name__ == "__main__":
    main()
