"""A/B helper for a kernel change: the headline model's embeddings (B = 256 and
B = 33, 80x200, bf16; every layer tap at B = 33) from two builds of the library
must be bitwise equal.  Each build runs in its own process (VOXEMB_LIB).

    python tools/lib_bitwise_check.py path/to/libvoxemb_old.so path/to/libvoxemb.so [model frames]

(model default res2net50_w24_s4_c32 at 200 frames; e.g. dpn68 600)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, model, frames):
    sys.path.insert(0, ROOT)
    import torch
    from bench import bench_features, weights_blob
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    blob = weights_blob(model, 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
    ex = Extractor(blob, device=0, precision="bf16")
    res = {}
    for n in ((256, 33) if frames <= 200 else (64, 7)):
        x = torch.from_numpy(bench_features(n, frames, 80, 0)).cuda()
        res[f"emb{n}"] = ex.run_device(x).cpu().numpy()
    taps, _ = ex.layer_outputs(torch.from_numpy(bench_features(5 if frames > 200 else 33, frames, 80, 1)).cuda())
    for i, t in enumerate(taps):
        res[f"tap{i}"] = np.asarray(t)
    torch.cuda.synchronize()
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3], int(sys.argv[4]))
        return 0
    model = sys.argv[3] if len(sys.argv) > 3 else "res2net50_w24_s4_c32"
    frames = sys.argv[4] if len(sys.argv) > 4 else "200"
    files = []
    for i, lib in enumerate(sys.argv[1:3]):
        out = f"/tmp/lib_bitwise_{i}.npz"
        env = dict(os.environ, VOXEMB_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, os.path.abspath(__file__), "--child", out, model, frames], env=env,
                       check=True)
        files.append(np.load(out))
    a, b = files
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    print(f"{len(a.files)} arrays compared; differing: {bad if bad else 'none'}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
