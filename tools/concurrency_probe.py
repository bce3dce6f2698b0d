"""Does splitting a step's batch over concurrent streams help?  Times the
headline forward (res2net50 80x200) as one handle on B utterances against
`--split` handles on B/split utterances each, every handle on its own stream,
all launched back to back per step (the kernels of the halves may co-run).

    python tools/concurrency_probe.py [--batch 256] [--split 2] [--steps 20]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="res2net50_w24_s4_c32")
    a = ap.parse_args()
    import torch
    import bench
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    blob = bench.weights_blob(a.model, 80, "/tmp/voxemb_cache")
    x = torch.from_numpy(bench.bench_features(a.batch, 200, 80)).to(dev)
    res = {}
    for split in [int(s) for s in a.splits.split(",")]:
        n = a.batch // split
        exs = [Extractor(blob, device=0) for _ in range(split)]
        streams = [torch.cuda.Stream(dev) for _ in range(split)]
        outs = [torch.empty((n, exs[0].dim), dtype=torch.float32, device=dev) for _ in range(split)]
        xs = [x[i * n:(i + 1) * n].contiguous() for i in range(split)]
        torch.cuda.synchronize()

        def step():
            for e, s, xi, o in zip(exs, streams, xs, outs):
                e.run_device(xi, o, s)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        res[f"split{split}"] = {"utt_per_s": round(a.batch * a.steps / el, 1),
                                "ms_per_step": round(el * 1e3 / a.steps, 3), "per_handle_batch": n}
        for e in exs:
            e.close()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
