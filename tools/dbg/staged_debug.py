import numpy as np, torch, os, sys
sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import synth, weights as W, archs
from voxsrc2020_speaker_verification_amd.extractor import Extractor
import bench
blob = bench.weights_blob("res2net50_w24_s4_c32", 80, "/tmp/voxemb_cache")
xs = [synth.make_features(4, 120, 80, seed=s) for s in (71, 72, 73)]
ex = Extractor(blob, 0, "bf16")
ref = [ex.run(x) for x in xs]
for mode in ("staged", "device"):
    for i, x in enumerate(xs):
        xt = torch.from_numpy(x).cuda()
        o = ex.run_device_staged(xt) if mode == "staged" else ex.run_device(xt)
        g = o.cpu().numpy()
        d = np.abs(g - ref[i]).max()
        print(mode, i, "maxdiff", d, "eq", np.array_equal(g, ref[i]), flush=True)
# replay on same buffers with new data, eager vs graph
os.environ["VOXEMB_NO_GRAPH"] = "1"
ex2 = Extractor(blob, 0, "bf16")
for i, x in enumerate(xs):
    g = ex2.run_device_staged(torch.from_numpy(x).cuda()).cpu().numpy()
    print("nograph staged", i, np.abs(g - ref[i]).max(), flush=True)
