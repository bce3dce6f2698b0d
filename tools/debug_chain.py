"""Fused split chain vs unfused branches: which path depends on batch position (GPU debug)."""
import io, os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
from voxsrc2020_speaker_verification_amd import archs, synth, weights
from voxsrc2020_speaker_verification_amd.extractor import Extractor
name, F, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
spec = archs.get_arch(name, F)
t = synth.make_weights(spec, calib_n=8, calib_T=120)
buf = io.BytesIO(); weights.save_blob(buf, spec, t); blob = buf.getvalue()
x = synth.make_features(3, T, F, seed=21)
res = {}
for cfg in ["", "NO_CHAIN", "NO_CHAIN+WIN_CIN=8", "NO_CHAIN+WIN_CIN=16", "NO_CHAIN+WIN_CIN=32", "NO_CHAIN+WIN_CIN=64"]:
    for k in ["VOXEMB_NO_CHAIN", "VOXEMB_NO_WIN", "VOXEMB_WIN_CIN"]:
        os.environ.pop(k, None)
    for k in cfg.split("+"):
        if k:
            k, _, v = k.partition("=")
            os.environ["VOXEMB_" + k] = v or "1"
    with Extractor(blob, 0, "bf16") as ex:
        full = ex.run(x)
        alone = [ex.run(x[i:i + 1])[0] for i in range(3)]
        pair = ex.run(x[1:3])
        open(f"gpurun_out/desc_{cfg or 'default'}.txt", "w").write("\n".join(ex.describe(torch.from_numpy(x[2:3]).cuda())))
    print(f"{cfg or 'default':16s}", [np.array_equal(full[i], alone[i]) for i in range(3)],
          "pair", [np.array_equal(pair[j], alone[j + 1]) for j in range(2)])
    res[cfg] = full
    print("   vs default:", [np.array_equal(full[i], res[""][i]) for i in range(3)])
