"""ORACLE (test infrastructure only) -- pure-Python restatement of Kaldi's
`apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300`
(tensorflow/tf_extract.py:63), and of Kaldi C++'s CompressedMatrix decode of
the `copy-feats --compress` arks that command reads (prepare_data.sh:69).
Kaldi is not vendored in the reference and is absent here, so the CMN is
restated from Kaldi's SlidingWindowCmnInternal
(feature-functions.cc; double-precision running sums updated by one frame at a
time, output = x + (-1/n) * sum): *parity unpinned* against Kaldi itself; it
pins the native implementation (csrc/kaldi_host.cpp) bit for bit.
"""

import numpy as np


def sliding_cmn(x, cmn_window=300, center=True, min_window=100):
    x = np.asarray(x, np.float32)
    T, F = x.shape
    xd = x.astype(np.float64)
    out = np.empty((T, F), np.float32)
    s = [0.0] * F
    last_start = last_end = -1
    for t in range(T):
        if center:
            ws = t - cmn_window // 2
            we = ws + cmn_window
        else:
            ws = t - cmn_window
            we = t + 1
        if ws < 0:
            we -= ws
            ws = 0
        if not center and we < min_window:
            we = min_window
        if we > T:
            ws -= we - T
            we = T
            if ws < 0:
                ws = 0
        if last_start == -1:
            for r in range(ws, we):
                row = xd[r]
                for f in range(F):
                    s[f] += row[f]
        else:
            if ws > last_start:
                row = xd[last_start]
                for f in range(F):
                    s[f] -= row[f]
            if we > last_end:
                row = xd[last_end]
                for f in range(F):
                    s[f] += row[f]
        n = we - ws
        last_start, last_end = ws, we
        alpha = -1.0 / n
        row = xd[t]
        out[t] = [row[f] + alpha * s[f] for f in range(F)]
    return out


def cm_decode_kaldi(blob):
    """Kaldi C++ CompressedMatrix::CopyToMat for the "CM " (one byte with column
    headers) format, from the bytes after "\\0BCM ": Uint16ToFloat =
    min + range * 1.52590218966964e-05f * v in float32, left to right;
    CharToFloat = p + (q - p) * v * (1/64.0 | 1/128.0 | 1/63.0) with the float32
    product promoted to double and the sum rounded to float32 once.  Parity
    unpinned against Kaldi (absent); pins vox_read_mat_kaldi bit for bit."""
    f32 = np.float32
    mn, rng = np.frombuffer(blob, f32, 2, 0)
    rows, cols = (int(v) for v in np.frombuffer(blob, np.int32, 2, 8))
    hdr = np.frombuffer(blob, np.uint16, 4 * cols, 16).reshape(cols, 4)
    data = np.frombuffer(blob, np.uint8, rows * cols, 16 + 8 * cols).reshape(cols, rows)
    out = np.empty((rows, cols), f32)
    c = f32(1.52590218966964e-05)
    for j in range(cols):
        p = [f32(mn + f32(rng * c) * f32(hdr[j, k])) for k in range(4)]
        for i in range(rows):
            v = int(data[j, i])
            if v <= 64:
                x = float(p[0]) + float(f32((p[1] - p[0]) * f32(v))) * (1 / 64.0)
            elif v <= 192:
                x = float(p[1]) + float(f32((p[2] - p[1]) * f32(v - 64))) * (1 / 128.0)
            else:
                x = float(p[2]) + float(f32((p[3] - p[2]) * f32(v - 192))) * (1 / 63.0)
            out[i, j] = f32(x)
    return out
