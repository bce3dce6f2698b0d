"""Per-tile phase timing of conv3x3_ks (the L3 w = 96 branches forming z_{k+1})
from its shader-clock stamps in the diagnostic build (conv3k.hip g_ks_trace:
workgroup 0 of the last z-forming launch, 12 waves x up to 16 tiles x 8 stamps).
Runs one B=256 80x200 forward of res2net50_w24_s4_c32 and prints, per wave, the
mean cycles of: DMA issue, K-half pass 1 (+ partial hand-off), pass 2, wait for
the x rows, barrier B, combine + epilogue + stores, wait + barrier D."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VOXEMB_LIB", os.path.join(ROOT, "voxsrc2020_speaker_verification_amd", "libvoxemb_diag.so"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from voxsrc2020_speaker_verification_amd import synth  # noqa: E402
from voxsrc2020_speaker_verification_amd import _native  # noqa: E402
from voxsrc2020_speaker_verification_amd.extractor import Extractor  # noqa: E402

blob = bench.weights_blob("res2net50_w24_s4_c32", 80, "/tmp/voxemb_cache")
ex = Extractor(blob, device=0, precision="bf16")
x = torch.from_numpy(synth.make_features(256, 200, 80, seed=1)).cuda()
out = torch.empty((256, ex.dim), dtype=torch.float32, device="cuda")
for _ in range(3):   # warm clocks; the stamps of the last forward remain
    ex.run_device(x, out, torch.cuda.current_stream())
torch.cuda.synchronize()
lib = _native.lib()
buf = np.zeros(12 * 16 * 8, dtype=np.uint64)
rc = lib.vox_debug_ks_trace(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes))
assert rc == 0, rc
tr = buf.reshape(12, 16, 8).astype(np.int64)
nt = int((tr[0, :, 0] > 0).sum())
t = tr[:, :nt]
names = ["issue", "pass1", "pass2", "xwait", "barB", "epi", "barD"]
print(f"tiles {nt}; workgroup 0 total {t[:, -1, 7].max() - t[:, 0, 0].min()} clk, "
      f"per tile {(t[0, -1, 7] - t[0, 0, 0]) / nt:.0f}")
print("wave  " + " ".join(f"{n:>7s}" for n in names) + "    next")
for w in range(12):
    d = [(t[w, :, i + 1] - t[w, :, i]).mean() for i in range(7)]
    nx = (t[w, 1:, 0] - t[w, :-1, 7]).mean() if nt > 1 else 0
    print(f"{w:4d}  " + " ".join(f"{v:7.0f}" for v in d) + f" {nx:7.0f}")
