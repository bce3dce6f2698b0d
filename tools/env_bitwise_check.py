"""A/B helper: the headline model's embeddings (33 utterances, 80x200, bf16)
with and without an environment switch must be bitwise equal.

    python tools/env_bitwise_check.py VOXEMB_SOME_SWITCH=1
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bench import weights_blob, bench_features
from voxsrc2020_speaker_verification_amd.extractor import Extractor

name, val = sys.argv[1].split("=", 1)
blob = weights_blob("res2net50_w24_s4_c32", 80, os.environ.get("VOXEMB_CACHE", "/tmp/voxemb_cache"))
x = torch.from_numpy(bench_features(33, 200, 80, 0)).cuda()
outs = []
for v in (None, val):
    if v is None:
        os.environ.pop(name, None)
    else:
        os.environ[name] = v
    ex = Extractor(blob, device=0, precision="bf16")
    outs.append(ex.run_device(x).cpu().numpy())
    torch.cuda.synchronize()
same = np.array_equal(outs[0], outs[1])
print(f"{name}={val} bitwise:", same, float(np.abs(outs[0] - outs[1]).max()))
sys.exit(0 if same else 1)
