"""Per-step phase timing of dpn_block_rows workgroup 0 (the last fused DPN68
stage-1 block of a forward) from its shader-clock stamps (VOXEMB_DPN_DBG=256,
diagnostic build).  Runs one B=64 80x600 dpn68 forward and prints, per wave,
the mean cycles of: 1x1a, barrier 1, grouped 3x3, barrier 2, staging of the
next input row, 1x1c, barrier 3, and the gap to the next step."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VOXEMB_LIB", os.path.join(ROOT, "voxsrc2020_speaker_verification_amd", "libvoxemb_diag.so"))
os.environ["VOXEMB_DPN_DBG"] = str(256 | int(os.environ.get("VOXEMB_DPN_DBG", "0")))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from voxsrc2020_speaker_verification_amd import synth  # noqa: E402
from voxsrc2020_speaker_verification_amd import _native  # noqa: E402
from voxsrc2020_speaker_verification_amd.extractor import Extractor  # noqa: E402

blob = bench.weights_blob("dpn68", 80, "/tmp/voxemb_cache")
ex = Extractor(blob, device=0, precision="bf16")
x = torch.from_numpy(synth.make_features(64, 600, 80, seed=1)).cuda()
out = torch.empty((64, ex.dim), dtype=torch.float32, device="cuda")
for _ in range(2):
    ex.run_device(x, out, torch.cuda.current_stream())
torch.cuda.synchronize()
lib = _native.lib()
buf = np.zeros(8 * 256 * 8, dtype=np.uint64)
rc = lib.vox_debug_dpn_trace(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes))
assert rc == 0, rc
tr = buf.reshape(8, 256, 8).astype(np.int64)
steps = int((tr[0, :, 0] > 0).sum())
t = tr[:, 2:steps - 2]   # steady state
print(f"steps {steps}; total {tr[0, steps - 1, 7] - tr[0, 0, 0]} clk, per step {(tr[0, steps - 1, 7] - tr[0, 0, 0]) / steps:.0f}")
names = ["1x1a", "bar1", "3x3", "bar2", "stage", "1x1c", "bar3"]
print("wave " + " ".join(f"{n:>7}" for n in names) + "     gap")
for w in range(8):
    d = [(t[w, :, i + 1] - t[w, :, i]).mean() for i in range(7)]
    gap = (t[w, 1:, 0] - t[w, :-1, 7]).mean()
    print(f"{w:4d} " + " ".join(f"{v:7.0f}" for v in d) + f" {gap:7.0f}")
