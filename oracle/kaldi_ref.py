"""ORACLE (test infrastructure only) -- pure-Python restatement of Kaldi's
`apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300`
(tensorflow/tf_extract.py:63), and of Kaldi C++'s CompressedMatrix decode of
the `copy-feats --compress` arks that command reads (prepare_data.sh:69),
and of the encoder that writes them (CompressedMatrix::CopyFromMat with
kAutomaticMethod, compressed-matrix.cc, restated from Kaldi's published
source; parity unpinned against Kaldi, pins vox_cm_compress_device).
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


def _u16(mn, rng, v):
    """FloatToUint16: float32 ratio, clamp to [0, 1], int(f * 65535 + 0.499)
    with the float32 product promoted to double."""
    f32 = np.float32
    f = f32(f32(f32(v) - mn) / rng)
    f = min(max(f, f32(0)), f32(1))
    return int(float(f32(f * f32(65535))) + 0.499)


def _char(p0, p25, p75, p100, v):
    """FloatToChar (float32 ratios, + 0.5 in double, truncate, clamp)."""
    f32 = np.float32
    if v < p25:
        a = int(float(f32(f32(f32(v - p0) / f32(p25 - p0)) * f32(64))) + 0.5)
        return min(max(a, 0), 64)
    if v < p75:
        a = 64 + int(float(f32(f32(f32(v - p25) / f32(p75 - p25)) * f32(128))) + 0.5)
        return min(max(a, 64), 192)
    a = 192 + int(float(f32(f32(f32(v - p75) / f32(p100 - p75)) * f32(63))) + 0.5)
    return min(max(a, 192), 255)


def cm_encode_kaldi(m):
    """Kaldi CompressedMatrix(mat, kAutomaticMethod) -> (token, payload bytes):
    "CM " (kSpeechFeature: per-column uint16 percentiles 0/25/75/100 at sorted
    positions 0, T/4, 3T/4, T-1 made strictly increasing, one byte per value,
    column-major) for rows > 8, else "CM2 " (kTwoByteAuto: uint16 row-major; Kaldi's
    WriteToken ends every token with a space, so the CM2 token is 4 bytes).
    Global header: min, max of the matrix (a constant matrix gets
    max = min + (1 + |min|)), range = max - min."""
    f32 = np.float32
    m = np.asarray(m, f32)
    rows, cols = m.shape
    mn = f32(m.min()) if m.size else f32(0)
    mx = f32(m.max()) if m.size else f32(0)
    if mx == mn:
        mx = f32(float(mn) + (1.0 + abs(float(mn))))
    rng = f32(mx - mn)
    head = np.array([mn, rng], f32).tobytes() + np.array([rows, cols], np.int32).tobytes()
    if rows <= 8:
        q = np.array([[_u16(mn, rng, m[i, j]) for j in range(cols)] for i in range(rows)],
                     np.uint16).reshape(rows, cols)
        return b"CM2 ", head + q.tobytes()   # WriteToken: "CM2" + " "
    c = f32(1.52590218966964e-05)
    hdrs, data = [], []
    q4 = rows // 4
    for j in range(cols):
        sd = np.sort(m[:, j])
        p0 = min(_u16(mn, rng, sd[0]), 65532)
        p25 = min(max(_u16(mn, rng, sd[q4]), p0 + 1), 65533)
        p75 = min(max(_u16(mn, rng, sd[3 * q4]), p25 + 1), 65534)
        p100 = max(_u16(mn, rng, sd[rows - 1]), p75 + 1)
        hdrs.append([p0, p25, p75, p100])
        pf = [f32(mn + f32(rng * c) * f32(v)) for v in (p0, p25, p75, p100)]
        data.append([_char(*pf, f32(m[i, j])) for i in range(rows)])
    return b"CM ", (head + np.array(hdrs, np.uint16).tobytes()
                    + np.array(data, np.uint8).tobytes())


def cm2_decode_kaldi(blob):
    """Kaldi CopyToMat for "CM2": min + v * float(range * (1 / 65535.0))."""
    f32 = np.float32
    mn, rng = np.frombuffer(blob, f32, 2, 0)
    rows, cols = (int(v) for v in np.frombuffer(blob, np.int32, 2, 8))
    q = np.frombuffer(blob, np.uint16, rows * cols, 16).reshape(rows, cols)
    inc = f32(float(rng) * (1.0 / 65535.0))
    return (mn + q.astype(f32) * inc).astype(f32)
