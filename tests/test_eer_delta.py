"""The metric's second half, "EER delta vs ref" (BASELINE.json), on what this
environment has: no VoxCeleb and no trained graph, so synthetic speakers --
each a fixed smooth spectral envelope, its utterances that envelope plus
independent noise -- through the same random-init Res2Net (well-conditioned,
synth.make_weights(residual_gain=0.25)) on three paths:

  * the product path: GPU bf16 (vox_embed),
  * the parity path: GPU fp32 (per layer within 1e-5 of the oracle, end to end
    within 1e-3: tests/test_gpu_parity.py, test_bf16_oracle.py),
  * the oracle side: the fp32 C++ restatement of the TF1 graph (oracle/cpu,
    within 1e-4 of oracle/models_ref.py), on a subset.

Trials are every same-speaker pair against every different-speaker pair;
scores are cosines of l2-normed embeddings and EER / minDCF come from
scoring.compute_eer_and_min_dcf (eer_minDCF.py:43-64, golden-exact).  The
numbers are printed as one JSON line (VOX_EER_OUT=path also writes them) --
profiles/r06_eer_delta.json holds the box run.  This pins how far bf16
moves the EER on a discriminative synthetic task; it is not the VoxCeleb1
EER of README.md:259-262 (unmeasurable here)."""

import io
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _speakers(S, U, T, F, seed):
    rng = np.random.default_rng(seed)
    k = np.exp(-0.5 * (np.arange(-6, 7) / 2.5) ** 2)
    k /= k.sum()
    env = np.stack([np.convolve(e, k, mode="same") for e in rng.standard_normal((S, F))]) * 3
    x = (env[:, None, None, :] + rng.standard_normal((S, U, T, F)) * 1.5).astype(np.float32)
    return x.reshape(S * U, T, F), np.repeat(np.arange(S), U)


def _eer(emb, lab):
    from voxsrc2020_speaker_verification_amd import scoring
    e = emb / np.linalg.norm(emb, axis=1, keepdims=True)
    iu = np.triu_indices(len(lab), 1)
    y = (lab[iu[0]] == lab[iu[1]]).astype(int)
    sc = (e @ e.T)[iu].astype(np.float64)
    eer, _, mindcf, _ = scoring.compute_eer_and_min_dcf(y, sc)
    return float(eer), float(mindcf), int(y.sum()), int(len(y) - y.sum()), sc


def test_eer_delta_bf16_vs_fp32_and_oracle():
    from oracle.cpu import CpuModel, build as cpu_build
    from voxsrc2020_speaker_verification_amd import archs, synth, weights
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    spec = archs.get_arch("res2net50_w24_s4_c32", 80)
    t = synth.make_weights(spec, seed=1, calib_n=8, calib_T=120, residual_gain=0.25)
    buf = io.BytesIO()
    weights.save_blob(buf, spec, t)
    blob = buf.getvalue()
    x, lab = _speakers(64, 16, 200, 80, seed=2020)             # 1,024 utterances
    with Extractor(blob, precision="bf16") as ex:
        e16 = ex.run(x)
    with Extractor(blob, precision="fp32") as ex:
        e32 = ex.run(x)
    r16, r32 = _eer(e16, lab), _eer(e32, lab)
    # the oracle side on a 256-utterance subset (16 speakers x 16)
    sub = np.isin(lab, np.arange(16))
    cpu_build.build()
    m = CpuModel(blob)
    ecpu = m.run(x[sub], threads=min(16, os.cpu_count() or 1))
    m.close()
    s32, scpu = _eer(e32[sub], lab[sub]), _eer(ecpu, lab[sub])
    s16 = _eer(e16[sub], lab[sub])
    res = {
        "task": "synthetic speakers (smooth spectral envelope + noise), res2net50_w24_s4_c32 "
                "80x200, random-init well-conditioned weights",
        "utterances": int(len(lab)), "target_trials": r16[2], "nontarget_trials": r16[3],
        "eer_gpu_bf16": r16[0], "eer_gpu_fp32": r32[0], "delta_eer_bf16_minus_fp32": r16[0] - r32[0],
        "mindcf_gpu_bf16": r16[1], "mindcf_gpu_fp32": r32[1],
        "score_max_abs_diff_bf16_fp32": float(np.abs(r16[4] - r32[4]).max()),
        "subset": {"utterances": int(sub.sum()), "eer_cpu_oracle_fp32": scpu[0],
                   "eer_gpu_fp32": s32[0], "eer_gpu_bf16": s16[0],
                   "score_max_abs_diff_gpu_fp32_vs_cpu": float(np.abs(s32[4] - scpu[4]).max())},
    }
    print(json.dumps(res))
    if os.environ.get("VOX_EER_OUT"):
        with open(os.environ["VOX_EER_OUT"], "w") as f:
            json.dump(res, f, indent=1)
    assert 0.0 < r32[0] < 0.25                        # the task discriminates
    assert res["subset"]["score_max_abs_diff_gpu_fp32_vs_cpu"] <= 1e-4
    assert scpu[0] == s32[0]                          # same trials -> same EER at fp32
    # bf16 against the fp32 path: within north_star's +-0.02 % absolute (box run:
    # -0.0016 %, profiles/r06_eer_delta.json; deterministic inputs and kernels)
    assert abs(r16[0] - r32[0]) <= 0.0002
