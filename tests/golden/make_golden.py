"""Generate the committed golden fixtures in tests/golden/ from the reference's
own importable modules (run in the build container, where /root/reference is
mounted; the fixtures travel, the reference does not).

    PYTHONDONTWRITEBYTECODE=1 KALDI_ROOT=/tmp python tests/golden/make_golden.py

What is pinned to what:
  * kaldi_io.py (tensorflow/kaldi_io.py)  -> FV record bytes (write_vec_flt
    :304-334), FM matrix bytes (write_mat), CM decode (_read_compressed_mat
    :471-504) on hand-built CM blobs, ark round trips (read_vec_flt_ark :249,
    read_mat_ark :367).
  * snorm.py (tensorflow/snorm.py)        -> l2norm / read_xvector / cohort
    speaker means / cosine trial scores / top-400 cohort mean,std / AS-norm
    (:23-131) on seeded synthetic embeddings; the `--weight_matrix` cohort
    (get_projection_weight :77-80) on a projection matrix this script pickles
    itself (its own file, loaded by the reference function as snorm.py does).
  * export_projection_weight.py:28-35 (imports TensorFlow, so not importable
    here): its post-read arithmetic -- swapaxes(-1,-2), reshape(-1, last),
    row l2norm with snorm's l2norm -- restated on a seeded head variable.
  * eer_minDCF.py                          -> compute_eer_and_min_dcf (:43-64).
  * utt2id.py                              -> read_spk / read_utt2spk (:20-41)
    and the argv pairing loop of its __main__ (:44-53), restated verbatim.
  * utils/split_scp.pl                     -> contiguous N-way shards
    (:211-244), by running the perl script.
Everything is small (seeded, a few hundred KB in total).
"""

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REF, "tensorflow"))
sys.path.insert(0, REF)
os.environ.setdefault("KALDI_ROOT", "/tmp")

import kaldi_io  # noqa: E402
import snorm  # noqa: E402
import eer_minDCF  # noqa: E402
import utt2id  # noqa: E402


def w(name, data):
    with open(os.path.join(OUT, name), "wb") as f:
        f.write(data)


def _bytes_via_file(writer):
    """kaldi_io's writers/readers need real binary file objects (fd.mode)."""
    fd, path = tempfile.mkstemp()
    os.close(fd)
    with open(path, "wb") as f:
        writer(f)
    with open(path, "rb") as f:
        return f.read(), path


def kaldi_fixtures():
    rng = np.random.default_rng(20201)
    # FV records
    vecs = {}
    for key, dim in (("utt-a", 256), ("spk1-utt_2", 3), ("x", 1), ("empty", 0)):
        vecs[key] = rng.standard_normal(dim).astype(np.float32)
    raw, path = _bytes_via_file(lambda f: [kaldi_io.write_vec_flt(f, v, k) for k, v in vecs.items()])
    w("fv_records.ark", raw)
    back = {k: v for k, v in kaldi_io.read_vec_flt_ark(path)}
    assert all(np.array_equal(back[k], vecs[k]) for k in vecs)
    np.savez(os.path.join(OUT, "fv_records.npz"), **{k.replace("-", "_"): v for k, v in vecs.items()})
    # FM matrices
    mats = {"m1": rng.standard_normal((7, 5)).astype(np.float32),
            "m2": (rng.standard_normal((30, 40)) * 10).astype(np.float32)}
    raw, path = _bytes_via_file(lambda f: [kaldi_io.write_mat(f, m, k) for k, m in mats.items()])
    w("fm_mats.ark", raw)
    back = {k: m for k, m in kaldi_io.read_mat_ark(path)}
    np.savez(os.path.join(OUT, "fm_mats.npz"), **back)
    # CM matrices: hand-built blobs, decoded by kaldi_io._read_compressed_mat
    cm_blobs = []
    for i, (rows, cols) in enumerate(((9, 4), (300, 80), (1, 3))):
        mn = np.float32(rng.uniform(-20, 0))
        rg = np.float32(rng.uniform(1, 40))
        hdr = np.sort(rng.integers(0, 65536, size=(cols, 4)), axis=1).astype(np.uint16)
        data = rng.integers(0, 256, size=(cols, rows)).astype(np.uint8)
        edge = [0, 64, 65, 192, 193, 255][:rows]
        data[0, :len(edge)] = edge
        blob = (b"\0BCM " + np.array([mn, rg], np.float32).tobytes() +
                np.array([rows, cols], np.int32).tobytes() + hdr.tobytes() + data.tobytes())
        cm_blobs.append(f"cm{i} ".encode() + blob)
    raw = b"".join(cm_blobs)
    w("cm_mats.ark", raw)
    cm_out = {k: np.asarray(m, np.float32)
              for k, m in kaldi_io.read_mat_ark(os.path.join(OUT, "cm_mats.ark"))}
    np.savez(os.path.join(OUT, "cm_mats.npz"), **cm_out)


def scoring_fixtures():
    rng = np.random.default_rng(7)
    D = 32
    tmp = tempfile.mkdtemp()
    # cohort: 450 speakers x 1-3 utterances, written as an FV ark
    spk2utt, cohort = {}, {}
    for s in range(450):
        spk = f"id{s:05d}"
        base = rng.standard_normal(D)
        utts = []
        for u in range(1 + s % 3):
            utt = f"{spk}/u{u}"
            cohort[utt] = (base + 0.5 * rng.standard_normal(D)).astype(np.float32)
            utts.append(utt)
        spk2utt[spk] = utts
    # one cohort utterance without a speaker (must be ignored) and one speaker
    # listing an utterance absent from the ark
    cohort["orphan/u0"] = rng.standard_normal(D).astype(np.float32)
    spk2utt["id00000"].append("id00000/missing")
    test = {f"t{i:03d}": rng.standard_normal(D).astype(np.float32) for i in range(40)}
    with open(os.path.join(OUT, "snorm_cohort.ark"), "wb") as f:
        for k, v in cohort.items():
            kaldi_io.write_vec_flt(f, v, k)
    with open(os.path.join(OUT, "snorm_test.ark"), "wb") as f:
        for k, v in test.items():
            kaldi_io.write_vec_flt(f, v, k)
    with open(os.path.join(OUT, "snorm_spk2utt"), "w") as f:
        for spk, utts in spk2utt.items():
            f.write(spk + " " + " ".join(utts) + "\n")
    keys = list(test)
    with open(os.path.join(OUT, "snorm_trials.txt"), "w") as f:
        for i in range(150):
            a, b = rng.choice(len(keys), 2, replace=False)
            f.write(f"{int(rng.integers(0, 2))} {keys[a]} {keys[b]}\n")
    tx = snorm.read_xvector(os.path.join(OUT, "snorm_test.ark"))
    cos = snorm.get_cosine_score(tx, os.path.join(OUT, "snorm_trials.txt"))
    coh = snorm.get_cohort_xvector(os.path.join(OUT, "snorm_cohort.ark"),
                                   os.path.join(OUT, "snorm_spk2utt"))
    mean, std = snorm.get_cohort_mean_std(tx, coh)
    asn = snorm.get_asnorm1_score(mean, std, cos)
    np.savez(os.path.join(OUT, "snorm_expected.npz"),
             cosine=np.array([s for _, _, s in cos], np.float64),
             asnorm=np.array([s for _, _, s in asn], np.float64),
             cohort_keys=np.array(list(coh)), cohort=np.array(list(coh.values())),
             mean=np.array([mean[k] for k in keys]), std=np.array([std[k] for k in keys]),
             test_keys=np.array(keys))


def projection_fixtures():
    """sc-CM style head variable [2, D, nspk] (two centres per speaker, kernel
    [..., in, out]) ->
    export_projection_weight.load's arithmetic -> pickle -> snorm's
    get_projection_weight -> top-400 cohort stats / AS-norm of the golden
    test set and trials."""
    rng = np.random.default_rng(31)
    D, nspk = 32, 230
    var = rng.standard_normal((2, D, nspk)).astype(np.float32)
    # export_projection_weight.py:28-35 (restated: the module imports TensorFlow)
    weight = np.swapaxes(var, -1, -2)
    weight = np.reshape(weight, (-1, weight.shape[-1]))
    weight = snorm.l2norm(weight, axis=1)
    fd, pkl = tempfile.mkstemp(suffix=".pkl")
    os.close(fd)
    import pickle
    with open(pkl, "wb") as f:
        pickle.dump(weight, f)                         # this script's own file
    coh = snorm.get_projection_weight(pkl)             # snorm.py:77-80
    tx = snorm.read_xvector(os.path.join(OUT, "snorm_test.ark"))
    cos = snorm.get_cosine_score(tx, os.path.join(OUT, "snorm_trials.txt"))
    mean, std = snorm.get_cohort_mean_std(tx, coh)
    asn = snorm.get_asnorm1_score(mean, std, cos)
    keys = list(tx)
    np.save(os.path.join(OUT, "proj_head_var.npy"), var)
    np.savez(os.path.join(OUT, "proj_expected.npz"), weight=weight,
             cohort=np.array(list(coh.values())), mean=np.array([mean[k] for k in keys]),
             std=np.array([std[k] for k in keys]),
             asnorm=np.array([s for _, _, s in asn], np.float64), test_keys=np.array(keys))


def eer_fixtures():
    rng = np.random.default_rng(11)
    cases = {}
    for name, n, ties in (("small", 200, False), ("ties", 500, True), ("large", 4000, False)):
        y = rng.integers(0, 2, size=n)
        s = rng.standard_normal(n) + 1.2 * y
        if ties:
            s = np.round(s, 1)
        eer, thr, mindcf, mthr = eer_minDCF.compute_eer_and_min_dcf(list(y), list(s), 1, 1, 0.01)
        cases[name] = dict(y=y.tolist(), s=s.tolist(), eer=float(eer), eer_threshold=float(thr),
                           min_dcf=float(mindcf), min_dcf_threshold=float(mthr))
    with open(os.path.join(OUT, "eer_cases.json"), "w") as f:
        json.dump(cases, f)


def utt2id_fixtures():
    tmp = tempfile.mkdtemp()
    p = lambda n: os.path.join(tmp, n)  # noqa: E731
    with open(p("utt2spk_a"), "w") as f:
        for i in range(30):
            f.write(f"spk{(i * 7) % 5}/u{i} spk{(i * 7) % 5}\n")
        f.write("ghost/u0 ghost\n")         # speaker not in the list -> skipped
    with open(p("spk_a"), "w") as f:
        f.write("\n".join(sorted({f"spk{i}" for i in range(5)})) + "\n")
    with open(p("utt2spk_b"), "w") as f:
        for i in range(10):
            f.write(f"B{i % 3}/x{i} B{i % 3}\n")
    with open(p("spk_b"), "w") as f:
        f.write("B0\nB1\nB2\n")
    files = {n: open(p(n)).read() for n in ("utt2spk_a", "spk_a", "utt2spk_b", "spk_b")}

    def main_loop(argv):  # utt2id.py:48-53 (__main__), restated verbatim
        assert len(argv) % 2 == 0
        out = {}
        for i in range(1, len(argv) // 2):
            out.update(utt2id.read_utt2spk(argv[i], utt2id.read_spk(argv[i + 1])))
        return out

    one = main_loop(["utt2id.py", p("utt2spk_a"), p("spk_a"), "out.pkl"])
    # two pairs: the reference pairs argv[i] with argv[i+1] for i in 1..n/2-1,
    # so the 2nd iteration reads spk_a as a utt2spk file -> ValueError
    try:
        main_loop(["utt2id.py", p("utt2spk_a"), p("spk_a"), p("utt2spk_b"), p("spk_b"), "out.pkl"])
        two = "no error"
    except Exception as e:  # noqa: BLE001
        two = type(e).__name__
    with open(os.path.join(OUT, "utt2id_cases.json"), "w") as f:
        json.dump({"files": files, "one_pair": one, "two_pairs_error": two}, f, indent=0)


def split_fixtures():
    cases = {}
    tmp = tempfile.mkdtemp()
    for n, N in ((10, 3), (8, 8), (17, 4), (5, 1), (100, 8)):
        src = os.path.join(tmp, f"in_{n}_{N}.scp")
        with open(src, "w") as f:
            for i in range(n):
                f.write(f"utt{i:04d} /data/feats.ark:{i * 100}\n")
        outs = [os.path.join(tmp, f"out_{n}_{N}_{k}.scp") for k in range(N)]
        subprocess.run(["perl", os.path.join(REF, "utils", "split_scp.pl"), src, *outs], check=True)
        cases[f"{n}_{N}"] = [[ln.split()[0] for ln in open(o)] for o in outs]
    with open(os.path.join(OUT, "split_scp_cases.json"), "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    kaldi_fixtures()
    scoring_fixtures()
    projection_fixtures()
    eer_fixtures()
    utt2id_fixtures()
    split_fixtures()
    print("golden fixtures written to", OUT)
