"""bf16 vs fp32-oracle cosine as a function of the BN-calibration batch used to
synthesise the weights (GPU experiment)."""
import io, os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from oracle import models_ref
from voxsrc2020_speaker_verification_amd import archs, synth, weights
from voxsrc2020_speaker_verification_amd.extractor import Extractor
name, F, T = "res2net50_w24_s4_c32", 80, 48
spec = archs.get_arch(name, F)
x = synth.make_features(4, T, F, seed=3)
cos = lambda a, b: np.sum(a * b, 1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
for cn, ct in ((4, 64), (16, 64), (64, 64), (64, 200)):
    t = synth.make_weights(spec, calib_n=cn, calib_T=ct)
    buf = io.BytesIO(); weights.save_blob(buf, spec, t)
    ref = models_ref.forward(spec, t, x)
    with Extractor(buf.getvalue(), 0, "bf16") as ex:
        got = ex.run(x)
    hv = t["batch_normalization_" + str(sum(1 for n in t if n.endswith("moving_variance")) - 2) + "/moving_variance"] if False else None
    print(f"calib_n={cn} calib_T={ct}: bf16 cos {cos(got, ref).round(5)}", flush=True)
