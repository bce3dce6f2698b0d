# first layer whose output for the same utterances differs between a big and a small batch
import numpy as np, os, sys, torch
sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import synth
from voxsrc2020_speaker_verification_amd.extractor import Extractor
import bench
model = sys.argv[1] if len(sys.argv) > 1 else "tdnn"
N, T, lo, hi = 700, 72, 690, 700
blob = bench.weights_blob(model, 80, "/tmp/voxemb_cache")
x = synth.make_features(N, T, 80, seed=12)
ex = Extractor(blob, 0, "bf16")
tb, eb = ex.layer_outputs(torch.from_numpy(x).cuda())
ts, es = ex.layer_outputs(torch.from_numpy(x[lo:hi]).cuda())
for i, (a, b) in enumerate(zip(tb, ts)):
    d = np.abs(a[lo:hi] - b)
    print(i, a.shape, "max diff", float(d.max()), "frac diff", float((d > 0).mean()), flush=True)
print("emb", float(np.abs(eb[lo:hi] - es).max()))
print("desc big:"); [print(" ", l[:120]) for l in ex.describe(torch.from_numpy(x).cuda())]
print("desc small:"); [print(" ", l[:120]) for l in ex.describe(torch.from_numpy(x[lo:hi]).cuda())]
