"""ORACLE (test infrastructure only) -- numpy restatement of the reference
TF1 inference graph for the extraction hot path, in two arithmetic modes.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may
import this module, and only as the checker / CPU baseline.  The product path
(`voxsrc2020_speaker_verification_amd`) never imports it.

Modes (the `precision` argument of `forward` / `layers`):
  * "fp32": the reference's own arithmetic (float32 variables and activations,
    models.py:191-197) -- the parity mode of the HIP library.
  * "bf16": the same graph with activations rounded to bfloat16
    (round-to-nearest-even) at exactly the points where the HIP library's bf16
    mode stores them (north_star: conv contractions on bf16 MFMA, fp32
    accumulation):
      - the input features (the stem / first TDNN layer read bf16 values);
      - conv weights (not BN statistics, not the fp32 head / attention weights);
      - every conv output after its epilogue: Res2Net stem / 1x1a / 3x3
        branch -> BN -> ReLU, the 1x1 projection -> BN, the 1x1c -> BN (+ the
        shortcut, then ReLU, one rounding), TDNN conv -> ReLU -> BN, DPN
        BN -> ReLU prologue of every conv input, DPN conv outputs, and the DPN
        residual sum r + conv (one rounding);
      - the Res2Net hierarchical addend z_k = x_k + y_{k-1} and the stride-2
        average pool of the last split;
      - stats pooling, attentive pooling and the head stay fp32 (they read the
        bf16 block output).
    BN is applied as (x - mean) * (1 / sqrt(var + eps)) in float32 with the
    BN and residual additions as separate roundings, as TF and the kernels do.

Parity status: TensorFlow is not installed and no frozen `.pb` exists in this
pipeline, so the model forward is *parity unpinned* against TF itself.  It is
re-derived from the reference source (cited per function below and in SURVEY.md
Appendix A) and cross-checked against an independent torch-CPU implementation
in `tests/test_oracle_models.py`.  The bf16 mode is pinned to the fp32 mode
(identical with rounding disabled) and to an independent float64-accumulation
run of itself (`tests/test_oracle_models.py`).

Layout is NHWC throughout, H = time, W = frequency (2-D models, expand_dim=3) or
W = 1, C = frequency (TDNN, expand_dim=2) -- tf_extract.py:32,
export_inference_graph.py:40-41.
"""

from __future__ import annotations

import numpy as np

BN_EPS_4D = 1.001e-5   # fused BN clamps eps to >= 1.001e-5 (models.py:62-67)
BN_EPS_2D = 1e-5       # 2-D head BNs are non-fused (models.py:20)
STATS_EPS = 1e-5       # stats_pool epsilon (models.py:262)

# float64 accumulation for every contraction (tests only: an independent
# summation order for the bf16 mode's self-check); default float32 BLAS
_ACC64 = False


def bf16(a):
    """Round float32 values to the nearest bfloat16 (ties to even), returned as
    float32 holding the bf16 value (what a bf16 store + reload gives)."""
    a = np.ascontiguousarray(a, np.float32)
    u = a.view(np.uint32)
    r = (u + (np.uint32(0x7FFF) + ((u >> np.uint32(16)) & np.uint32(1)))) & np.uint32(0xFFFF0000)
    return r.view(np.float32)


class _Q:
    """Rounding points of one arithmetic mode (module docstring)."""

    def __init__(self, precision):
        if precision not in ("fp32", "bf16"):
            raise ValueError(precision)
        self.bf = precision == "bf16"

    def act(self, x):
        return bf16(x) if self.bf else np.asarray(x, np.float32)

    def w(self, k):
        return bf16(k) if self.bf else k


def _mm(a, b):
    if _ACC64:
        return (a.astype(np.float64) @ b.astype(np.float64)).astype(np.float32)
    return (a @ b).astype(np.float32)


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
        if kh == kw == 1 and sh == sw == 1:
            cols = xg.reshape(N * Ho * Wo, cig)
        else:
            taps = []
            for ky in range(kh):
                for kx in range(kw):
                    y0, x0 = ky * dh, kx * dw
                    taps.append(xg[:, y0:y0 + (Ho - 1) * sh + 1:sh, x0:x0 + (Wo - 1) * sw + 1:sw, :])
            cols = np.stack(taps, axis=3).reshape(N * Ho * Wo, kh * kw * cig)
        wg = w[..., g * cog:(g + 1) * cog].reshape(kh * kw * cig, cog)
        outs.append(_mm(cols, wg).reshape(N, Ho, Wo, cog))
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


def batch_norm_2d(x, mean, var, eps):
    """The 2-D head BNs: tf.compat.v1.layers.batch_normalization picks the fused
    kernel only for 4-D inputs, so on the [N, D] head TF1 runs
    tf.nn.batch_normalization, x * inv + (-mean * inv) with inv = rsqrt(var +
    eps) (offset and scale None: center=False, scale=False), as a Mul and an
    Add -- two float32 roundings.  inv here is the correctly rounded 1/sqrt;
    TF's Eigen rsqrt (EIGEN_FAST_MATH) may differ in the last bit (TF absent:
    unpinned)."""
    inv = (np.float32(1.0) / np.sqrt(var.astype(np.float32) + np.float32(eps))).astype(np.float32)
    nmi = (-mean.astype(np.float32) * inv).astype(np.float32)
    return ((x.astype(np.float32) * inv).astype(np.float32) + nmi).astype(np.float32)


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
    x = batch_norm_2d(x, t[bn1 + "/moving_mean"], t[bn1 + "/moving_variance"], BN_EPS_2D)
    x = (x @ t[dense]).astype(np.float32)
    return batch_norm_2d(x, t[bn2 + "/moving_mean"], t[bn2 + "/moving_variance"], BN_EPS_2D)


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


def _head_layer(p):
    """stats already pooled + flattened -> BN(2-D) -> dense -> BN(2-D), fp32."""
    m1, v1 = p.bn()
    dense = p.conv()
    m2, v2 = p.bn()
    assert p.done()

    def f(x):
        x = batch_norm_2d(x, m1, v1, BN_EPS_2D)
        x = _mm(x, dense)
        return batch_norm_2d(x, m2, v2, BN_EPS_2D)
    return f


def tdnn_layers(spec, tensors, q):
    """tdnn_model.py:128-155 with conv_relu_bn_block :24-30.  Layer 0 takes the
    [N,T,F] features (expand_dim 2 -> [N,T,1,F], tf_extract.py:32)."""
    p = _Params(tensors)
    out = []
    for i, (k, d) in enumerate(zip(spec["kernels"], spec["dilations"])):
        w = q.w(p.conv())
        m, v = p.bn()

        def f(x, w=w, d=d, m=m, v=v, first=(i == 0)):
            if first:
                x = q.act(np.asarray(x, np.float32)[:, :, None, :])
            return q.act(batch_norm(relu(conv2d_same(x, w, (1, 1), (d, 1))), m, v))
        out.append((f"tdnn{i}", f))
    hd = _head_layer(p)
    out.append(("pool+head", lambda x: hd(flatten_nhwc(stats_pool(x)))))
    return out


def res2net_split_conv(h, kernel, bns, stride, split, width, q=None):
    """res2net_model.py:26-78 (hierarchical split-scale 3x3 conv); `h` is the
    (rounded) 1x1a output, kernel the (rounded) [3,3,w,w*(split-1)] variable."""
    q = q or _Q("fp32")
    if stride > 1:
        h = np.pad(h, ((0, 0), (1, 1), (1, 1), (0, 0)))       # fixed_padding(k=3)
    parts = [h[..., i * width:(i + 1) * width] for i in range(split)]
    kernels = [kernel[..., i * width:(i + 1) * width] for i in range(split - 1)]

    def cbr(inp, k, bn):
        if stride == 1:
            y = conv2d_same(inp, k)
        else:
            y = conv2d(inp, k, (stride, stride))                # VALID
        return q.act(relu(batch_norm(y, *bn)))

    outs = [cbr(parts[0], kernels[0], bns[0])]
    for idx in range(1, split - 1):
        inp = parts[idx]
        if stride == 1:
            inp = q.act(inp + outs[idx - 1])
        outs.append(cbr(inp, kernels[idx], bns[idx]))
    if stride == 1:
        outs.append(parts[split - 1])
    else:
        outs.append(q.act(avg_pool3x3s2_valid(parts[split - 1])))
    return np.concatenate(outs, axis=3)


def res2net_layers(spec, tensors, q):
    """res2net_model.py:185-243 (v1 bottleneck :81-103, block_layer :106-136).
    Layer 0 (the stem) takes the [N,T,F] features (expand_dim 3 -> [N,T,F,1])."""
    p = _Params(tensors)
    s = spec["split"]
    ws = q.w(p.conv())
    bs = p.bn()

    def stem(x):                                              # :192-203
        x = q.act(np.asarray(x, np.float32)[..., None])
        return q.act(relu(batch_norm(conv2d_fixed_padding(x, ws, 1), *bs)))
    out = [("stem", stem)]
    for i, nblocks in enumerate(spec["block_sizes"]):
        w = spec["widths"][i]
        for b in range(nblocks):
            stride = spec["block_strides"][i] if b == 0 else 1
            proj = (q.w(p.conv()), p.bn()) if b == 0 else None
            ka, bna = q.w(p.conv()), p.bn()
            kern = q.w(p.conv())
            bns = [p.bn() for _ in range(s - 1)]
            kc, bnc = q.w(p.conv()), p.bn()

            def block(x, stride=stride, proj=proj, ka=ka, bna=bna, kern=kern, bns=bns, kc=kc,
                      bnc=bnc, w=w):
                if proj is not None:                          # projection_shortcut
                    sc = q.act(batch_norm(conv2d_fixed_padding(x, proj[0], stride), *proj[1]))
                else:
                    sc = x
                h = q.act(relu(batch_norm(conv2d_fixed_padding(x, ka, 1), *bna)))
                h = res2net_split_conv(h, kern, bns, stride, s, w, q)
                h = batch_norm(conv2d_fixed_padding(h, kc, 1), *bnc)
                return q.act(relu(h + sc))
            out.append((f"layer{i + 1}.block{b}", block))
    if spec.get("pool") == "att":                            # res2net_model.py:229
        k1, k2 = p.conv(), p.conv()
        pool = lambda x: flatten_nhwc(att_stats_pool(x, k1, k2))
    else:
        pool = lambda x: flatten_nhwc(stats_pool(x))
    hd = _head_layer(p)
    out.append(("pool+head", lambda x: hd(pool(x))))
    return out


def dpn_layers(spec, tensors, q):
    """dpn_model.py:111-168 (dual_path_block :57-87, bn_relu_conv :40-45).
    Each block maps the concatenated state [res | dense] (a channel prefix of
    one stage buffer in the HIP plan) to the next state."""
    from voxsrc2020_speaker_verification_amd.archs import dpn_stage_params  # spec helper only
    p = _Params(tensors)
    G = spec["cardinality"]

    def bnrelu_args():
        return p.bn()

    def bn_relu(t, bn):
        return q.act(relu(batch_norm(t, *bn)))

    ws = q.w(p.conv())
    bs = p.bn()

    def stem(x):                                              # conv_bn_relu :32-37
        x = q.act(np.asarray(x, np.float32)[..., None])
        return q.act(relu(batch_norm(conv2d_same(x, ws), *bs)))
    out = [("stem", stem)]
    for si, (bw, r, inc, blocks, ptype) in enumerate(dpn_stage_params(spec)):
        for b in range(blocks):
            stride = 2 if (b == 0 and ptype == "downsampled") else 1
            pr = (bnrelu_args(), q.w(p.conv())) if b == 0 else None
            c1 = (bnrelu_args(), q.w(p.conv()))
            c2 = (bnrelu_args(), q.w(p.conv()))
            c3 = (bnrelu_args(), q.w(p.conv()))

            def block(inp, stride=stride, pr=pr, c1=c1, c2=c2, c3=c3, bw=bw):
                if pr is not None:
                    proj = q.act(conv2d_same(bn_relu(inp, pr[0]), pr[1], (stride, stride)))
                    r0, d0 = proj[..., :bw], proj[..., bw:]
                else:
                    r0, d0 = inp[..., :bw], inp[..., bw:]
                h = q.act(conv2d_same(bn_relu(inp, c1[0]), c1[1]))
                h = q.act(conv2d_same(bn_relu(h, c2[0]), c2[1], (stride, stride), groups=G))
                h = conv2d_same(bn_relu(h, c3[0]), c3[1])
                return np.concatenate([q.act(r0 + h[..., :bw]), d0, q.act(h[..., bw:])], axis=3)
            out.append((f"stage{si + 1}.block{b}", block))
    fb = p.bn()
    hd = _head_layer(p)
    # concat_bn_relu :24-29, stats pool, head
    out.append(("pool+head", lambda x: hd(flatten_nhwc(stats_pool(bn_relu(x, fb))))))
    return out


def _eps_from(spec):
    global BN_EPS_4D, BN_EPS_2D
    BN_EPS_4D = float(spec.get("bn_eps_4d", 1.001e-5))
    BN_EPS_2D = float(spec.get("bn_eps_2d", 1e-5))


def layers(spec, tensors, precision="fp32"):
    """The forward as [(name, fn)]: fn maps one layer's input to its output;
    the first takes the [N,T,F] features, the last ("pool+head") returns the
    [N,D] embeddings.  The boundaries are the block outputs the HIP plan
    exposes as taps (vox_debug_taps), so a test can feed layer i the GPU's own
    output of layer i-1 (teacher forcing)."""
    _eps_from(spec)
    q = _Q(precision)
    fam = spec["family"]
    if fam == "tdnn":
        return tdnn_layers(spec, tensors, q)
    if fam == "res2net":
        return res2net_layers(spec, tensors, q)
    if fam == "dpn":
        return dpn_layers(spec, tensors, q)
    raise ValueError(fam)


def forward(spec, tensors, feats, precision="fp32"):
    """One `sess.run(outputs, {inputs: x})` (tf_extract.py:108).

    feats: [N, T, F] float32 (post-CMN FBANK).  The expand_dim rule of
    tf_extract.py:32 is applied by the first layer: TDNN -> [N,T,1,F],
    2-D -> [N,T,F,1]."""
    x = np.asarray(feats, np.float32)
    for _, f in layers(spec, tensors, precision):
        x = f(x)
    return x


def embed_utterance(spec, tensors, feat, max_frames=1000, precision="fp32"):
    """tf_extract.py:96-111 chunk rule: n = 1 + (T-25)//1000; chunk i has
    length 1000 if (i+1)*1000 <= T else T-1000*i; length-weighted average.
    T < 25 gives 0 chunks and a ZeroDivisionError, as in the reference."""
    T = feat.shape[0]
    n = 1 + (T - 25) // max_frames
    vals, lens = [], []
    for i in range(n):
        L = max_frames if (i + 1) * max_frames <= T else T - i * max_frames
        e = forward(spec, tensors, feat[None, i * max_frames:i * max_frames + L], precision)
        vals.append(e * L)
        lens.append(L)
    return (sum(vals) / sum(lens))[0]
