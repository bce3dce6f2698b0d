"""Fused bottleneck vs unfused (VOXEMB_NO_BNECK) on one model: which settings differ (GPU debug)."""
import io, os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import archs, synth, weights
from voxsrc2020_speaker_verification_amd.extractor import Extractor
name, F, T, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
spec = archs.get_arch(name, F)
t = synth.make_weights(spec, calib_n=8, calib_T=120)
buf = io.BytesIO(); weights.save_blob(buf, spec, t); blob = buf.getvalue()
x = synth.make_features(N, T, F, seed=21)
def run(env):
    for k in ["VOXEMB_NO_BNECK", "VOXEMB_BNECK_NSEG"]:
        os.environ.pop(k, None)
    os.environ.update(env)
    with Extractor(blob, 0, "bf16") as ex:
        return ex.run(x)
ref = run({"VOXEMB_NO_BNECK": "1"})
for ns in ["1", "2", "3", "8", "25"]:
    got = run({"VOXEMB_BNECK_NSEG": ns})
    d = np.abs(got - ref).max(1)
    print(f"nseg={ns:3s} equal={np.array_equal(got, ref)} maxdiff per utt={d}", flush=True)
