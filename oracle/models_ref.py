"""ORACLE (test infrastructure only) -- numpy fp32 restatement of the reference
TF1 inference graph for the extraction hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker / CPU baseline.  The product path
(`voxsrc2020_speaker_verification_amd`) never imports it.

Parity status: TensorFlow is not installed and no frozen `.pb` exists in this
pipeline, so the model forward is *parity unpinned* against TF itself.  It is
re-derived from the reference source (cited per function below and in SURVEY.md
Appendix A) and cross-checked against an independent torch-CPU implementation
in `tests/test_oracle_models.py`.

Layout is NHWC throughout, H = time, W = frequency (2-D models, expand_dim=3) or
W = 1, C = frequency (TDNN, expand_dim=2) -- tf_extract.py:32,
export_inference_graph.py:40-41.
"""

from __future__ import annotations

import numpy as np

BN_EPS_4D = 1.001e-5   # fused BN clamps eps to >= 1.001e-5 (models.py:62-67)
BN_EPS_2D = 1e-5       # 2-D head BNs are non-fused (models.py:20)
STATS_EPS = 1e-5       # stats_pool epsilon (models.py:262)


# --------------------------------------------------------------------------- ops

def tf_same_pads(n, k, s, d=1):
    """TF 'SAME' padding (before, after) for one spatial dim."""
    keff = (k - 1) * d + 1
    out = -(-n // s)
    total = max((out - 1) * s + keff - n, 0)
    return total // 2, total - total // 2


def conv2d(x, w, strides=(1, 1), dilations=(1, 1), pads=((0, 0), (0, 0)), groups=1):
    """tf.nn.conv2d NHWC with explicit (top,bottom),(left,right) zero pads, VALID
    afterwards.  `w` is HWIO [kh, kw, cin/groups, cout] (models.py:191-203).
    Grouped conv follows the per-group split formulation the reference keeps
    for CPU (models.py:205-218)."""
    x = np.asarray(x, np.float32)
    N, H, W, C = x.shape
    kh, kw, cig, cout = w.shape
    sh, sw = strides
    dh, dw = dilations
    (pt, pb), (pl, pr) = pads
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    Hp, Wp = H + pt + pb, W + pl + pr
    Ho = (Hp - ((kh - 1) * dh + 1)) // sh + 1
    Wo = (Wp - ((kw - 1) * dw + 1)) // sw + 1
    assert C == cig * groups and cout % groups == 0
    cog = cout // groups
    outs = []
    for g in range(groups):
        xg = xp[..., g * cig:(g + 1) * cig]
        taps = []
        for ky in range(kh):
            for kx in range(kw):
                y0, x0 = ky * dh, kx * dw
                taps.append(xg[:, y0:y0 + (Ho - 1) * sh + 1:sh, x0:x0 + (Wo - 1) * sw + 1:sw, :])
        cols = np.stack(taps, axis=3).reshape(N * Ho * Wo, kh * kw * cig)
        wg = w[..., g * cog:(g + 1) * cog].reshape(kh * kw * cig, cog)
        outs.append((cols @ wg).reshape(N, Ho, Wo, cog))
    return np.concatenate(outs, axis=3) if groups > 1 else outs[0]


def conv2d_same(x, w, strides=(1, 1), dilations=(1, 1), groups=1):
    """padding='SAME' (TF semantics, asymmetric when needed -- Appendix A.2/A.4)."""
    kh, kw = w.shape[:2]
    ph = tf_same_pads(x.shape[1], kh, strides[0], dilations[0])
    pw = tf_same_pads(x.shape[2], kw, strides[1], dilations[1])
    return conv2d(x, w, strides, dilations, (ph, pw), groups)


def conv2d_fixed_padding(x, w, stride):
    """models.py:155-168: SAME when stride 1, else fixed_padding (:107-152) +
    VALID.  fixed pad for k: beg=(k-1)//2, end=(k-1)-beg."""
    k = w.shape[0]
    if stride == 1:
        return conv2d_same(x, w)
    pb = (k - 1) // 2
    pe = (k - 1) - pb
    return conv2d(x, w, (stride, stride), (1, 1), ((pb, pe), (pb, pe)))


def batch_norm(x, mean, var, eps=None):
    """Inference BN with no gamma/beta (center=False, scale=False): models.py:62-67.
    eps defaults to the 4-D (fused) epsilon of the current blob."""
    if eps is None:
        eps = BN_EPS_4D
    inv = (np.float32(1.0) / np.sqrt(var.astype(np.float32) + np.float32(eps))).astype(np.float32)
    return ((x - mean.astype(np.float32)) * inv).astype(np.float32)


def relu(x):
    return np.maximum(x, np.float32(0))


def avg_pool3x3s2_valid(x):
    """tf.nn.avg_pool2d(ksize=3, strides=2, 'VALID') (res2net_model.py:77)."""
    N, H, W, C = x.shape
    Ho, Wo = (H - 3) // 2 + 1, (W - 3) // 2 + 1
    acc = np.zeros((N, Ho, Wo, C), np.float32)
    for ky in range(3):
        for kx in range(3):
            acc += x[:, ky:ky + 2 * (Ho - 1) + 1:2, kx:kx + 2 * (Wo - 1) + 1:2, :]
    return (acc / np.float32(9.0)).astype(np.float32)


def stats_pool(x, eps=STATS_EPS):
    """models.py:262-269: tf.nn.moments over H (two-pass, population var),
    std = sqrt(var + eps), concat [mean, std] on C -> [N, 1, W, 2C]."""
    mean = x.mean(axis=1, keepdims=True, dtype=np.float32)
    var = np.square(x - mean).mean(axis=1, keepdims=True, dtype=np.float32)
    std = np.sqrt(var + np.float32(eps)).astype(np.float32)
    return np.concatenate([mean, std], axis=3).astype(np.float32)


def att_stats_pool(x, k1, k2, eps=STATS_EPS):
    """models.py:273-303 (att_with_mean_std=True): moments over H, att input =
    concat[x, tile(mean), tile(std)] on C, logits = conv1x1(tanh(conv1x1(.)))
    (no bias), softmax over H, weighted mean and sqrt(E_w[x^2] - mean^2 + eps).
    x: [N,H,W,C] -> [N,1,W,2C]."""
    m = stats_pool(x, eps)                                   # [N,1,W,2C]
    tiled = np.broadcast_to(m, x.shape[:3] + (m.shape[3],))
    a = np.concatenate([x, tiled], axis=3).astype(np.float32)
    h = np.tanh(a @ k1[0, 0]).astype(np.float32)
    logits = (h @ k2[0, 0]).astype(np.float32)
    z = logits - logits.max(axis=1, keepdims=True)
    e = np.exp(z).astype(np.float32)
    w = (e / e.sum(axis=1, keepdims=True)).astype(np.float32)
    wm = (x * w).sum(axis=1, keepdims=True, dtype=np.float32)
    wss = (x * x * w).sum(axis=1, keepdims=True, dtype=np.float32)
    ws = np.sqrt(wss - wm * wm + np.float32(eps)).astype(np.float32)
    return np.concatenate([wm, ws], axis=3).astype(np.float32)


def flatten_nhwc(x):
    """tf.compat.v1.layers.flatten on NHWC: feature index = (h*W + w)*C + c."""
    return x.reshape(x.shape[0], -1)


def head(x, t, names):
    """BN(2-D) -> dense (no bias) -> BN(2-D) -> 'outputs'
    (res2net_model.py:239-242, tdnn_model.py:148-153, dpn_model.py:163-167)."""
    bn1, dense, bn2 = names
    x = batch_norm(x, t[bn1 + "/moving_mean"], t[bn1 + "/moving_variance"], BN_EPS_2D)
    x = (x @ t[dense]).astype(np.float32)
    return batch_norm(x, t[bn2 + "/moving_mean"], t[bn2 + "/moving_variance"], BN_EPS_2D)


# ----------------------------------------------------------------- backbones

class _Params:
    """Consumes blob tensors strictly in manifest (creation) order."""

    def __init__(self, tensors):
        self.items = list(tensors.items())
        self.i = 0

    def conv(self):
        name, a = self.items[self.i]
        assert name.endswith("/kernel"), name
        self.i += 1
        return a

    def bn(self):
        (n1, m), (n2, v) = self.items[self.i], self.items[self.i + 1]
        assert n1.endswith("moving_mean") and n2.endswith("moving_variance"), (n1, n2)
        self.i += 2
        return m, v

    def done(self):
        return self.i == len(self.items)


def _head_tail(p, x):
    m1, v1 = p.bn()
    x = batch_norm(x, m1, v1, BN_EPS_2D)
    x = (x @ p.conv()).astype(np.float32)
    m2, v2 = p.bn()
    assert p.done()
    return batch_norm(x, m2, v2, BN_EPS_2D)


def tdnn_forward(spec, tensors, x):
    """tdnn_model.py:128-155 with conv_relu_bn_block :24-30.  x: [N,T,1,F]."""
    p = _Params(tensors)
    for k, d in zip(spec["kernels"], spec["dilations"]):
        w = p.conv()
        x = conv2d_same(x, w, (1, 1), (d, 1))
        x = relu(x)
        m, v = p.bn()
        x = batch_norm(x, m, v)
    x = flatten_nhwc(stats_pool(x))
    return _head_tail(p, x)


def res2net_split_conv(h, kernel, bns, stride, split, width):
    """res2net_model.py:26-78 (hierarchical split-scale 3x3 conv)."""
    if stride > 1:
        h = np.pad(h, ((0, 0), (1, 1), (1, 1), (0, 0)))       # fixed_padding(k=3)
    parts = [h[..., i * width:(i + 1) * width] for i in range(split)]
    kernels = [kernel[..., i * width:(i + 1) * width] for i in range(split - 1)]

    def cbr(inp, k, bn):
        if stride == 1:
            y = conv2d_same(inp, k)
        else:
            y = conv2d(inp, k, (stride, stride))                # VALID
        return relu(batch_norm(y, *bn))

    outs = [cbr(parts[0], kernels[0], bns[0])]
    for idx in range(1, split - 1):
        inp = parts[idx]
        if stride == 1:
            inp = inp + outs[idx - 1]
        outs.append(cbr(inp, kernels[idx], bns[idx]))
    if stride == 1:
        outs.append(parts[split - 1])
    else:
        outs.append(avg_pool3x3s2_valid(parts[split - 1]))
    return np.concatenate(outs, axis=3)


def res2net_forward(spec, tensors, x):
    """res2net_model.py:185-243 (v1 bottleneck :81-103, block_layer :106-136).
    x: [N,T,F,1]."""
    p = _Params(tensors)
    s = spec["split"]
    x = conv2d_fixed_padding(x, p.conv(), 1)                 # :192-194
    x = relu(batch_norm(x, *p.bn()))                         # :202-203
    for i, nblocks in enumerate(spec["block_sizes"]):
        w = spec["widths"][i]
        for b in range(nblocks):
            stride = spec["block_strides"][i] if b == 0 else 1
            if b == 0:
                sc = batch_norm(conv2d_fixed_padding(x, p.conv(), stride), *p.bn())
            else:
                sc = x
            h = relu(batch_norm(conv2d_fixed_padding(x, p.conv(), 1), *p.bn()))
            kern = p.conv()
            bns = [p.bn() for _ in range(s - 1)]
            h = res2net_split_conv(h, kern, bns, stride, s, w)
            h = batch_norm(conv2d_fixed_padding(h, p.conv(), 1), *p.bn())
            x = relu(h + sc)
    if spec.get("pool") == "att":                            # res2net_model.py:229
        x = flatten_nhwc(att_stats_pool(x, p.conv(), p.conv()))
    else:
        x = flatten_nhwc(stats_pool(x))
    return _head_tail(p, x)


def dpn_forward(spec, tensors, x):
    """dpn_model.py:111-168 (dual_path_block :57-87, bn_relu_conv :40-45).
    x: [N,T,F,1]."""
    from voxsrc2020_speaker_verification_amd.archs import dpn_stage_params  # spec helper only
    p = _Params(tensors)
    G = spec["cardinality"]

    def bn_relu(t):
        return relu(batch_norm(t, *p.bn()))

    x = relu(batch_norm(conv2d_same(x, p.conv()), *p.bn()))    # conv_bn_relu :32-37
    state = x
    for bw, r, inc, blocks, ptype in dpn_stage_params(spec):
        for b in range(blocks):
            stride = 2 if (b == 0 and ptype == "downsampled") else 1
            if b == 0:
                inp = state if not isinstance(state, list) else np.concatenate(state, axis=3)
                proj = conv2d_same(bn_relu(inp), p.conv(), (stride, stride))
                r0, d0 = proj[..., :bw], proj[..., bw:]
            else:
                r0, d0 = state
                inp = np.concatenate(state, axis=3)
            h = conv2d_same(bn_relu(inp), p.conv())
            h = conv2d_same(bn_relu(h), p.conv(), (stride, stride), groups=G)
            h = conv2d_same(bn_relu(h), p.conv())
            state = [r0 + h[..., :bw], np.concatenate([d0, h[..., bw:]], axis=3)]
    x = bn_relu(np.concatenate(state, axis=3))                  # concat_bn_relu :24-29
    x = flatten_nhwc(stats_pool(x))
    return _head_tail(p, x)


def _eps_from(spec):
    global BN_EPS_4D, BN_EPS_2D
    BN_EPS_4D = float(spec.get("bn_eps_4d", 1.001e-5))
    BN_EPS_2D = float(spec.get("bn_eps_2d", 1e-5))


def forward(spec, tensors, feats):
    """One `sess.run(outputs, {inputs: x})` (tf_extract.py:108).

    feats: [N, T, F] float32 (post-CMN FBANK).  The expand_dim rule of
    tf_extract.py:32 is applied here: TDNN -> [N,T,1,F], 2-D -> [N,T,F,1]."""
    feats = np.asarray(feats, np.float32)
    _eps_from(spec)
    fam = spec["family"]
    if fam == "tdnn":
        return tdnn_forward(spec, tensors, feats[:, :, None, :])
    if fam == "res2net":
        return res2net_forward(spec, tensors, feats[..., None])
    if fam == "dpn":
        return dpn_forward(spec, tensors, feats[..., None])
    raise ValueError(fam)


def embed_utterance(spec, tensors, feat, max_frames=1000):
    """tf_extract.py:96-111 chunk rule: n = 1 + (T-25)//1000; chunk i has
    length 1000 if (i+1)*1000 <= T else T-1000*i; length-weighted average.
    T < 25 gives 0 chunks and a ZeroDivisionError, as in the reference."""
    T = feat.shape[0]
    n = 1 + (T - 25) // max_frames
    vals, lens = [], []
    for i in range(n):
        L = max_frames if (i + 1) * max_frames <= T else T - i * max_frames
        e = forward(spec, tensors, feat[None, i * max_frames:i * max_frames + L])
        vals.append(e * L)
        lens.append(L)
    return (sum(vals) / sum(lens))[0]
