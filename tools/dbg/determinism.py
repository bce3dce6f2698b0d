# which kernel makes the forward non-deterministic at a small batch (n=4, T=120)?
import numpy as np, os, sys
sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import synth
from voxsrc2020_speaker_verification_amd.extractor import Extractor
import bench
blob = bench.weights_blob("res2net50_w24_s4_c32", 80, "/tmp/voxemb_cache")
N, T = int(sys.argv[1]), int(sys.argv[2])
x = synth.make_features(N, T, 80, seed=71)
x2 = synth.make_features(N, T, 80, seed=72)
sw = ["", "VOXEMB_NO_GEMM_WIDE", "VOXEMB_NO_BNECK", "VOXEMB_NO_CHAIN_FUSED", "VOXEMB_NO_S2_FUSED",
      "VOXEMB_NO_CONV3_RW", "VOXEMB_NO_CONV3_UTT", "VOXEMB_NO_CONV3_S2R", "VOXEMB_NO_STEM", "VOXEMB_NO_NW",
      "VOXEMB_NO_GEMM_PIPE"]
for s in sw:
    for k in sw[1:]:
        os.environ.pop(k, None)
    if s:
        os.environ[s] = "1"
    ex = Extractor(blob, 0, "bf16")
    a = ex.run(x)
    ex.run(x2)
    b = ex.run(x)
    # the same input after a different one: any difference is state carried over
    per = np.abs(a - b).max(axis=1)
    print(f"{s or 'default':24s} x, x2, x: max diff per utterance {np.round(per, 3).tolist()}", flush=True)
    ex.close()
