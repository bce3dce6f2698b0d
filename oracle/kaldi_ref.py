"""ORACLE (test infrastructure only) -- pure-Python restatement of Kaldi's
`apply-cmvn-sliding --norm-vars=false --center=true --cmn-window=300`
(tensorflow/tf_extract.py:63).  Kaldi is not vendored in the reference and is
absent here, so this is restated from Kaldi's SlidingWindowCmnInternal
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
