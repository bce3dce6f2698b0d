"""Per-step phase timing of bneck_fused block 0 from its shader-clock stamps
(VOXEMB_BNECK_DBG=256; diagnostics).  Runs one B=256 80x200 forward of
res2net50_w24_s4_c32 and prints, per wave, the mean cycles of: phase 0 work,
wait at barrier 1, phase 1 work, wait at barrier 2 (the last bneck launch)."""
import ctypes as C
import os
import sys

import numpy as np

os.environ.setdefault("VOXEMB_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "voxsrc2020_speaker_verification_amd", "libvoxemb_diag.so"))
os.environ["VOXEMB_BNECK_DBG"] = str(256 | int(os.environ.get("VOXEMB_BNECK_DBG", "0")))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
ex.run_device(x, out, torch.cuda.current_stream())
torch.cuda.synchronize()
lib = _native.lib()
buf = np.zeros(8 * 512 * 4, dtype=np.uint64)
rc = lib.vox_debug_bneck_trace(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes))
assert rc == 0, rc
tr = buf.reshape(8, 512, 4).astype(np.int64)
steps = int((tr[0, :, 0] > 0).sum())
t = tr[:, :steps]
print(f"steps {steps}; total {(t[0, -1, 3] - t[0, 0, 0])} clk")
for w in range(8):
    p0 = (t[w, :, 1] - t[w, :, 0]).mean()
    b1 = (t[w, :, 2] - t[w, :, 1]).mean()
    p1 = (t[w, :, 3] - t[w, :, 2]).mean()
    b2 = (t[w, 1:, 0] - t[w, :-1, 3]).mean()
    if int(os.environ.get("VOXEMB_BNECK_DBG", "0")) & 2048:
        # stamp 1 exists only on the 1x1c waves' steps that own an output row
        ok = t[w, :, 1] > t[w, :, 0]
        if ok.any():
            p0 = (t[w, ok, 1] - t[w, ok, 0]).mean()
            b1 = (t[w, ok, 2] - t[w, ok, 1]).mean()
        else:
            p0, b1 = 0.0, (t[w, :, 2] - t[w, :, 0]).mean()
        print(f"wave {w}: residual wait {p0:7.0f}  phase-0 work {b1:7.0f}  res issue+barrier1 {p1:7.0f}  "
              f"phase 1 + barrier 2 {b2:7.0f}  ({int(ok.sum())} owning steps)")
    elif int(os.environ.get("VOXEMB_BNECK_DBG", "0")) & 1024:
        print(f"wave {w}: phase0 {p0:7.0f}  barrier1+staging {b1:7.0f}  chain MFMA loop {p1:7.0f}  "
              f"epilogue+barrier2 {b2:7.0f}")
    else:
        print(f"wave {w}: phase0 {p0:7.0f}  wait1 {b1:7.0f}  phase1 {p1:7.0f}  wait2 {b2:7.0f}")
