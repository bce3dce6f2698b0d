"""Backbone specifications and the tensor manifest each one consumes.

The reference defines its backbones as module-level callables that build a TF1
graph; the frozen `.pb` then carries the variables in creation order.  Here a
backbone is a small dict of hyper-parameters, and :func:`manifest` lists the
tensors (name, shape, kind) in exactly the order the reference creates them, so
that a weight blob is just those tensors back to back.  The native executor
(`csrc/plan.cpp`) walks the same order.

Reference configs:
  * tdnn                      -- tensorflow/models/tdnn_model.py:158-161
  * res2net50_w24_s4_c32      -- tensorflow/models/res2net_model.py:252-256
  * res2net50_w24_s4_c64      -- res2net_model.py:246-250
  * res2net50_w8_s6_c16       -- res2net_model.py:258-262
  * dpn68                     -- tensorflow/models/dpn_model.py:171

TF variable naming follows the reference scopes (`conv2d`, `conv2d_1`, ...,
`batch_normalization_k`, `dense`), which is what a `.pb` converter will see.
"""

from __future__ import annotations

import copy

# BatchNorm epsilons (Appendix A.6 of SURVEY.md):
#  * 4-D BNs go through tf.nn.fused_batch_norm, which clamps eps to >= 1.001e-5
#    (models.py:62-67 passes 1e-5; TF1 keras normalization `_fused_batch_norm`).
#  * 2-D head BNs are non-fused and keep eps = 1e-5 (models.py:20).
BN_EPS_4D = 1.001e-5
BN_EPS_2D = 1e-5
STATS_POOL_EPS = 1e-5  # models.py:262

ARCHS = {
    # tdnn_model.py:158-161 -- 5 x [conv(k,1) dilated SAME -> ReLU -> BN]
    "tdnn": dict(family="tdnn", filters=[512, 512, 512, 512, 1536],
                 kernels=[5, 3, 3, 1, 1], dilations=[1, 2, 3, 1, 1],
                 output_dim=256, expand_dim=2),
    # res2net_model.py:252-256
    "res2net50_w24_s4_c32": dict(family="res2net", num_filters=[32, 64, 128, 256],
                                 widths=[24, 48, 96, 192], block_sizes=[3, 4, 6, 3],
                                 block_strides=[1, 2, 2, 2], split=4, output_dim=256,
                                 expand_dim=3),
    # res2net_model.py:246-250
    "res2net50_w24_s4_c64": dict(family="res2net", num_filters=[64, 128, 256, 512],
                                 widths=[24, 48, 96, 192], block_sizes=[3, 4, 6, 3],
                                 block_strides=[1, 2, 2, 2], split=4, output_dim=256,
                                 expand_dim=3),
    # res2net_model.py:258-262
    "res2net50_w8_s6_c16": dict(family="res2net", num_filters=[16, 32, 64, 128],
                                widths=[8, 16, 32, 64], block_sizes=[3, 4, 6, 3],
                                block_strides=[1, 2, 2, 2], split=6, output_dim=192,
                                expand_dim=3),
    # res2net_model.py:264-280 -- deeper Res2Nets with attentive statistics
    # pooling (models.py:273-303, att_dim 128, attention over [x, mean, std])
    "res2net101_w24_s4_c32_att": dict(family="res2net", num_filters=[32, 64, 128, 256],
                                      widths=[24, 48, 96, 192], block_sizes=[3, 4, 23, 3],
                                      block_strides=[1, 2, 2, 2], split=4, output_dim=256,
                                      expand_dim=3, pool="att", att_dim=128),
    "res2net152_w24_s4_c32_att": dict(family="res2net", num_filters=[32, 64, 128, 256],
                                      widths=[24, 48, 96, 192], block_sizes=[3, 8, 36, 3],
                                      block_strides=[1, 2, 2, 2], split=4, output_dim=256,
                                      expand_dim=3, pool="att", att_dim=128),
    "res2net200_w24_s4_c32_att": dict(family="res2net", num_filters=[32, 64, 128, 256],
                                      widths=[24, 48, 96, 192], block_sizes=[3, 24, 36, 3],
                                      block_strides=[1, 2, 2, 2], split=4, output_dim=256,
                                      expand_dim=3, pool="att", att_dim=128),
    # dpn_model.py:171 (num_init_features=10, k_r=128, G=32, k_sec, inc_sec)
    "dpn68": dict(family="dpn", num_init_features=10, k_r=128, bw=64, cardinality=32,
                  k_sec=[3, 4, 12, 3], inc_sec=[16, 32, 32, 64], output_dim=256,
                  expand_dim=3),
}


def get_arch(name: str, feat_dim: int, **overrides) -> dict:
    """Return a full spec (a copy) for backbone `name` at `feat_dim` mel bins."""
    if name not in ARCHS:
        raise KeyError(f"unknown backbone {name!r}; known: {sorted(ARCHS)}")
    spec = copy.deepcopy(ARCHS[name])
    spec["name"] = name
    spec["feat_dim"] = int(feat_dim)
    spec.update(overrides)
    return spec


class _Namer:
    """TF1 unique-name counters for default-named scopes/layers."""

    def __init__(self):
        self.counts = {}

    def __call__(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"


def _bn(out, namer, c, kind="bn4", prefix=""):
    name = prefix + namer("batch_normalization")
    out.append((name + "/moving_mean", (c,), kind))
    out.append((name + "/moving_variance", (c,), kind))


def _conv(out, namer, shape):
    out.append((namer("conv2d") + "/kernel", tuple(shape), "conv"))


def pooled_dim(spec: dict) -> int:
    """Feature count after stats-pool + flatten (input to the head)."""
    fam = spec["family"]
    if fam == "tdnn":
        return 2 * spec["filters"][-1]
    w = spec["feat_dim"]
    if fam == "res2net":
        for s in spec["block_strides"]:
            w = (w + s - 1) // s
        return w * 2 * spec["num_filters"][-1] * 4
    if fam == "dpn":
        # stages 2..4 downsample by 2 (TF SAME: ceil)
        for _ in range(3):
            w = (w + 1) // 2
        return w * 2 * dpn_out_channels(spec)
    raise ValueError(fam)


def dpn_stage_params(spec: dict):
    """(bw, r, inc, blocks, projection_type) per stage -- dpn_model.py:135-157."""
    stages = []
    types = ["projected", "downsampled", "downsampled", "downsampled"]
    for i, mult in enumerate([1, 2, 4, 8]):
        bw = spec["bw"] * mult
        r = spec["k_r"] * bw // spec["bw"]
        stages.append((bw, r, spec["inc_sec"][i], spec["k_sec"][i], types[i]))
    return stages


def dpn_out_channels(spec: dict) -> int:
    c = None
    for bw, r, inc, blocks, _ in dpn_stage_params(spec):
        dense = 2 * inc + blocks * inc
        c = bw + dense
    return c


def manifest(spec: dict):
    """List of (name, shape, kind) in reference creation order.

    kind: "conv" (HWIO kernel), "dense" ([in,out]), "bn4"/"bn2" (moving stats).
    """
    fam = spec["family"]
    out = []
    namer = _Namer()
    F = spec["feat_dim"]
    if fam == "tdnn":
        cin = F
        for cout, k in zip(spec["filters"], spec["kernels"]):
            _conv(out, namer, (k, 1, cin, cout))
            _bn(out, namer, cout)
            cin = cout
    elif fam == "res2net":
        s = spec["split"]
        nf0 = spec["num_filters"][0]
        _conv(out, namer, (3, 3, 1, nf0))           # res2net_model.py:192-194
        _bn(out, namer, nf0)                        # :202
        cin = nf0
        for i, nblocks in enumerate(spec["block_sizes"]):
            nf, w = spec["num_filters"][i], spec["widths"][i]
            cout = 4 * nf
            for b in range(nblocks):
                if b == 0:                          # projection_shortcut :125-127
                    _conv(out, namer, (1, 1, cin, cout))
                    _bn(out, namer, cout)
                _conv(out, namer, (1, 1, cin, s * w))   # conv1x1a :89
                _bn(out, namer, s * w)
                scope = namer("conv2d")             # res2net_pad_conv_bn_relu :30
                out.append((scope + "/kernel", (3, 3, w, w * (s - 1)), "conv"))
                inner = _Namer()
                for _ in range(s - 1):
                    _bn(out, inner, w, prefix=scope + "/")
                _conv(out, namer, (1, 1, s * w, cout))  # conv1x1c :98
                _bn(out, namer, cout)
                cin = cout
        if spec.get("pool") == "att":              # att_stats_pool, models.py:288-291
            A = spec["att_dim"]
            out.append(("att_stats_pool/conv2d/kernel", (1, 1, 3 * cin, A), "conv"))
            out.append(("att_stats_pool/conv2d_1/kernel", (1, 1, A, cin), "conv"))
    elif fam == "dpn":
        G = spec["cardinality"]
        c0 = spec["num_init_features"]
        _conv(out, namer, (3, 3, 1, c0))            # conv_bn_relu stem :113
        _bn(out, namer, c0)
        res_c, dense_c = c0, 0                      # stem output is a plain tensor
        for bw, r, inc, blocks, ptype in dpn_stage_params(spec):
            for b in range(blocks):
                cin = res_c + dense_c
                if b == 0:                          # projected / downsampled :75-80
                    _bn(out, namer, cin)
                    _conv(out, namer, (1, 1, cin, bw + 2 * inc))
                    res_c, dense_c = bw, 2 * inc
                _bn(out, namer, cin)                # bn_relu_conv_layers :48-54
                _conv(out, namer, (1, 1, cin, r))
                _bn(out, namer, r)
                _conv(out, namer, (3, 3, r // G, r))
                _bn(out, namer, r)
                _conv(out, namer, (1, 1, r, bw + inc))
                dense_c += inc                      # concat(inputs1, inputs_1) :87
        _bn(out, namer, res_c + dense_c)            # concat_bn_relu :152
    else:
        raise ValueError(f"unknown family {fam!r}")
    # head: BN(2-D) -> dense (no bias) -> BN(2-D)   e.g. res2net_model.py:239-241
    D = pooled_dim(spec)
    _bn(out, namer, D, kind="bn2")
    out.append(("dense/kernel", (D, spec["output_dim"]), "dense"))
    _bn(out, namer, spec["output_dim"], kind="bn2")
    return out


def param_count(spec: dict, include_head=True) -> int:
    n = 0
    for name, shape, kind in manifest(spec):
        if kind in ("conv", "dense") and (include_head or kind == "conv"):
            p = 1
            for d in shape:
                p *= d
            n += p
    return n
