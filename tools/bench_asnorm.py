"""Time vox_asnorm_stats at the VoxCeleb1 scale of SURVEY.md §8 a16
(153,516 trials x 5,994 cohort means x 256) against the numpy restatement on
a row sample.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import scoring as S  # noqa: E402


def main():
    n, m, d, k = 153516, 5994, 256, 400
    rng = np.random.default_rng(0)
    t = rng.standard_normal((n, d)).astype(np.float32)
    t /= np.linalg.norm(t, axis=1, keepdims=True)
    c = rng.standard_normal((m, d)).astype(np.float32)
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    trial = {i: v for i, v in enumerate(t)}
    cohort = {i: v for i, v in enumerate(c)}
    S.cohort_mean_std_gpu({0: t[0]}, cohort)            # warm-up (library load)
    t0 = time.perf_counter()
    mg, sg = S.cohort_mean_std_gpu(trial, cohort, topk=k)
    gpu_s = time.perf_counter() - t0
    ns = 4096
    sample = {i: t[i] for i in range(ns)}
    t0 = time.perf_counter()
    mc, sc = S.cohort_mean_std(sample, cohort, topk=k)
    cpu_s = (time.perf_counter() - t0) * n / ns
    err = max(abs(mg[i] - mc[i]) for i in range(ns))
    print(json.dumps({"trials": n, "cohort": m, "dim": d, "topk": k,
                      "gpu_s": round(gpu_s, 4), "cpu_numpy_s_extrapolated": round(cpu_s, 2),
                      "cpu_sample_rows": ns, "max_abs_mean_diff": float(err)}))


if __name__ == "__main__":
    main()
