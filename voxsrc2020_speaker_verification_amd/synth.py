"""Synthetic weights and features (there are no checkpoints or VoxCeleb data here).

* Kernels follow TF1 `variance_scaling_initializer()` defaults used by every
  reference conv/dense (models.py:191-197, :306-309): scale 1, fan_in,
  truncated normal (stddev = sqrt(1/fan_in)/0.8796..., cut at 2 sigma).
* BN moving statistics are calibrated once by a training-mode pass on seeded
  features, so activations are O(1) and reduced-precision error is realistic.
  The calibration pass is an independent torch-CPU implementation of the
  backbones (NCHW, `F.conv2d` with explicit TF pads); the tests also use it as
  the second implementation that cross-checks the numpy oracle.

Features: `numpy.random.default_rng(seed).standard_normal` (post-CMN FBANK is
roughly zero-mean), SURVEY.md §8(d).
"""

from __future__ import annotations

import math

import numpy as np

from . import archs

_TRUNC_STD = 0.87962566103423978


def make_features(n, T, F, seed=0):
    return np.random.default_rng(seed).standard_normal((n, T, F), dtype=np.float32)


def _trunc_normal(rng, shape, std):
    out = rng.standard_normal(shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * std).astype(np.float32)


def init_weights(spec, seed=1):
    rng = np.random.default_rng(seed)
    t = {}
    for name, shape, kind in archs.manifest(spec):
        if kind in ("conv", "dense"):
            fan_in = int(np.prod(shape[:-1]))
            t[name] = _trunc_normal(rng, shape, math.sqrt(1.0 / fan_in) / _TRUNC_STD)
        elif name.endswith("moving_mean"):
            t[name] = np.zeros(shape, np.float32)
        else:
            t[name] = np.ones(shape, np.float32)
    return t


# --------------------------------------------------------- torch CPU backbones

class _TorchParams:
    def __init__(self, tensors, calibrate):
        import torch
        self.torch = torch
        self.tensors = tensors
        self.names = list(tensors)
        self.i = 0
        self.calibrate = calibrate

    def conv(self):
        name = self.names[self.i]
        self.i += 1
        return self.torch.from_numpy(np.ascontiguousarray(self.tensors[name]))

    def bn(self, x, eps, gain=None):
        """Inference BN; in calibration mode first set the moving stats to the
        batch statistics of `x` (per channel over N,H,W; or over N for 2-D),
        the variance divided by gain**2 when a gain is given."""
        torch = self.torch
        nm, nv = self.names[self.i], self.names[self.i + 1]
        self.i += 2
        dims = (0, 2, 3) if x.dim() == 4 else (0,)
        if self.calibrate:
            xd = x.double()
            m = xd.mean(dim=dims)
            v = ((xd - m.view((1, -1) + (1,) * (x.dim() - 2))) ** 2).mean(dim=dims)
            if gain is not None:
                v = v / (gain * gain)
            self.tensors[nm] = m.float().numpy()
            self.tensors[nv] = v.float().numpy()
        m = torch.from_numpy(self.tensors[nm])
        v = torch.from_numpy(self.tensors[nv])
        shape = (1, -1) + (1,) * (x.dim() - 2)
        return (x - m.view(shape)) * torch.rsqrt(v + eps).view(shape)


def _tf_pads(n, k, s, d=1):
    keff = (k - 1) * d + 1
    out = -(-n // s)
    total = max((out - 1) * s + keff - n, 0)
    return total // 2, total - total // 2


def _conv(x, w_hwio, stride=1, dil=(1, 1), pads=None, groups=1, same=True):
    """x: NCHW; w: HWIO numpy-derived torch tensor."""
    import torch.nn.functional as F
    w = w_hwio.permute(3, 2, 0, 1).contiguous()
    kh, kw = w.shape[2], w.shape[3]
    if pads is None:
        if same:
            ph = _tf_pads(x.shape[2], kh, stride, dil[0])
            pw = _tf_pads(x.shape[3], kw, stride, dil[1])
        else:
            ph = pw = (0, 0)
    else:
        ph, pw = pads
    x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
    return F.conv2d(x, w, stride=stride, dilation=dil, groups=groups)


def _stats_pool(x, eps):
    import torch
    mean = x.mean(dim=2, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=2, keepdim=True)
    y = torch.cat([mean, torch.sqrt(var + eps)], dim=1)   # [N, 2C, 1, W]
    return y.permute(0, 2, 3, 1).reshape(x.shape[0], -1)   # NHWC flatten


def _att_stats_pool(x, k1, k2, eps):
    """models.py:273-303 on NCHW: attention logits from [x, mean, std] (tiled
    over T), softmax over T, weighted mean / std per (channel, frequency)."""
    import torch
    mean = x.mean(dim=2, keepdim=True)
    var = ((x - mean) ** 2).mean(dim=2, keepdim=True)
    ms = torch.cat([mean, torch.sqrt(var + eps)], dim=1).expand(-1, -1, x.shape[2], -1)
    h = torch.tanh(_conv(torch.cat([x, ms], dim=1), k1))
    w = torch.softmax(_conv(h, k2), dim=2)
    wm = (x * w).sum(dim=2, keepdim=True)
    wss = (x * x * w).sum(dim=2, keepdim=True)
    y = torch.cat([wm, torch.sqrt(wss - wm * wm + eps)], dim=1)
    return y.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def torch_forward(spec, tensors, feats, calibrate=False, residual_gain=None):
    """Independent torch-CPU forward (fp32).  With calibrate=True the BN moving
    statistics in `tensors` are overwritten by batch statistics, in order;
    residual_gain scales the calibrated Res2Net residual branches (the 1x1c
    BN) so the synthetic network is well-conditioned (see make_weights)."""
    import torch
    import torch.nn.functional as F
    e4, e2 = archs.BN_EPS_4D, archs.BN_EPS_2D
    p = _TorchParams(tensors, calibrate)
    x = torch.from_numpy(np.ascontiguousarray(feats, dtype=np.float32))
    fam = spec["family"]
    with torch.no_grad():
        if fam == "tdnn":
            x = x.permute(0, 2, 1).unsqueeze(3)           # [N, F, T, 1]
            for k, d in zip(spec["kernels"], spec["dilations"]):
                x = F.relu(_conv(x, p.conv(), 1, (d, 1)))
                x = p.bn(x, e4)
        elif fam == "res2net":
            s = spec["split"]
            x = x.unsqueeze(1)                            # [N, 1, T, F]
            x = F.relu(p.bn(_conv(x, p.conv()), e4))
            for i, nblocks in enumerate(spec["block_sizes"]):
                w = spec["widths"][i]
                for b in range(nblocks):
                    st = spec["block_strides"][i] if b == 0 else 1
                    if b == 0:
                        sc = p.bn(_conv(x, p.conv(), st, same=(st == 1)), e4)
                    else:
                        sc = x
                    h = F.relu(p.bn(_conv(x, p.conv()), e4))
                    kern = p.conv()
                    if st > 1:
                        h = F.pad(h, (1, 1, 1, 1))
                    parts = torch.split(h, w, dim=1)
                    outs = []
                    for j in range(s - 1):
                        inp = parts[j]
                        if st == 1 and j > 0:
                            inp = inp + outs[-1]
                        kj = kern[..., j * w:(j + 1) * w]
                        y = _conv(inp, kj, st, same=(st == 1))
                        outs.append(F.relu(p.bn(y, e4)))
                    if st == 1:
                        outs.append(parts[s - 1])
                    else:
                        outs.append(F.avg_pool2d(parts[s - 1], 3, st))
                    h = torch.cat(outs, dim=1)
                    h = p.bn(_conv(h, p.conv()), e4, residual_gain)
                    x = F.relu(h + sc)
        elif fam == "dpn":
            G = spec["cardinality"]
            x = x.unsqueeze(1)
            x = F.relu(p.bn(_conv(x, p.conv()), e4))
            state = x
            for bw, r, inc, blocks, ptype in archs.dpn_stage_params(spec):
                for b in range(blocks):
                    st = 2 if (b == 0 and ptype == "downsampled") else 1
                    if b == 0:
                        inp = state if not isinstance(state, list) else torch.cat(state, 1)
                        proj = _conv(F.relu(p.bn(inp, e4)), p.conv(), st)
                        r0, d0 = proj[:, :bw], proj[:, bw:]
                    else:
                        r0, d0 = state
                        inp = torch.cat(state, 1)
                    h = _conv(F.relu(p.bn(inp, e4)), p.conv())
                    h = _conv(F.relu(p.bn(h, e4)), p.conv(), st, groups=G)
                    h = _conv(F.relu(p.bn(h, e4)), p.conv())
                    state = [r0 + h[:, :bw], torch.cat([d0, h[:, bw:]], 1)]
            x = F.relu(p.bn(torch.cat(state, 1), e4))
        else:
            raise ValueError(fam)
        if spec.get("pool") == "att":
            x = _att_stats_pool(x, p.conv(), p.conv(), archs.STATS_POOL_EPS)
        else:
            x = _stats_pool(x, archs.STATS_POOL_EPS)
        x = p.bn(x, e2)
        x = x @ p.conv()
        x = p.bn(x, e2)
    assert p.i == len(p.names)
    return x.numpy()


def make_weights(spec, seed=1, calib_n=16, calib_T=200, calib_seed=12345, residual_gain=None):
    """Variance-scaling init + one BN calibration pass.

    With plain calibration a random-init Res2Net is chaotic: an fp32 input
    perturbation of 1e-3 already moves embeddings to cosine ~0.98, and bf16
    rounding to ~0.85 (DESIGN.md "Precision").  residual_gain (e.g. 0.25)
    damps every residual branch during calibration, giving a well-conditioned
    network (as trained ones are) on which bf16-vs-fp32 checks discriminate."""
    t = init_weights(spec, seed)
    feats = make_features(calib_n, calib_T, spec["feat_dim"], calib_seed)
    torch_forward(spec, t, feats, calibrate=True, residual_gain=residual_gain)
    return t
