"""The device side of the extraction reader (vox_cm_chunks_device: "CM "
payloads decoded, sliding-CMN'd and gathered into the padded chunk batch on
the GPU) against the host reader (vox_read_chunks(_ragged): Kaldi C++ CM
arithmetic + the double-precision CMN recursion) -- bitwise, batch by batch
and end to end through the streaming extractor.  tf_extract.py:63 (the
apply-cmvn-sliding pipe over prepare_data.sh:69's `copy-feats --compress`
arks).  CM arks written with the oracle's Kaldi encoder (oracle/kaldi_ref.py)."""

import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cm_ark(tmp_path, lens, seed, F=80):
    from oracle.kaldi_ref import cm_encode_kaldi
    from voxsrc2020_speaker_verification_amd.frontend import format_cm_record
    rng = np.random.default_rng(seed)
    ark, scp = str(tmp_path / "cm.ark"), str(tmp_path / "cm.scp")
    with open(ark, "wb") as fa, open(scp, "w") as fs:
        for i, T in enumerate(lens):
            m = (rng.standard_normal((int(T), F)) * 3 + rng.standard_normal(F) * 4).astype(np.float32)
            tok, payload = cm_encode_kaldi(m)
            assert tok == b"CM "
            rec, off = format_cm_record(f"u{i:03d}", np.frombuffer(payload, np.uint8), int(T))
            pos = fa.tell()
            fa.write(rec)
            fs.write(f"u{i:03d} {ark}:{pos + off}\n")
    return scp


LENS = [25, 26, 300, 301, 449, 450, 999, 1000, 1001, 1149, 1150, 1151, 2100, 2999, 3100, 40, 612, 77]


@pytest.mark.parametrize("ragged,cmn", [(True, True), (False, True), (True, False)])
def test_device_batches_equal_host_batches(tmp_path, ragged, cmn):
    import torch
    from voxsrc2020_speaker_verification_amd import kaldi, stream
    from voxsrc2020_speaker_verification_amd._native import check, lib
    table = stream.ChunkTable(kaldi.read_scp(_cm_ark(tmp_path, LENS, 3)), threads=4)
    assert table.cm_device_ok()
    F = table.feat_dim
    _, batches = stream.plan_batches(table.T, 5, ragged=ragged)
    dev = torch.device("cuda", 0)
    for b in batches:
        L, items = b[0], b[1]
        lens = b[2] if ragged else [L] * len(items)
        n = len(items)
        host = np.zeros(n * L * F, np.float32)
        if ragged:
            table.read_ragged(items, lens, L, host, cmn)
        else:
            table.read(items, L, host, cmn)
        utts, meta, nbytes, total, mx = table.cm_batch(items, lens, cmn)
        blob = np.zeros(nbytes, np.uint8)
        table.read_cm_payloads(utts, meta, blob)
        d_blob = torch.from_numpy(blob).to(dev)
        d_meta = torch.from_numpy(meta).to(dev)
        work = torch.empty(2 * total * F, dtype=torch.float32, device=dev)
        out = torch.full((n * L * F,), float("nan"), dtype=torch.float32, device=dev)
        check(lib().vox_cm_chunks_device(C.c_void_p(d_blob.data_ptr()), C.c_void_p(d_meta.data_ptr()),
                                         len(utts), total, mx, n, L, F, 300 if cmn else 0,
                                         C.c_void_p(work.data_ptr()), C.c_void_p(out.data_ptr()), None))
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), host.view(np.uint32)), (L, lens)


@pytest.mark.parametrize("name,lanes", [("res2net50_w24_s4_c32", 2), ("tdnn", 1)])
def test_extraction_device_reader_equals_host_reader(weights, tmp_path, name, lanes):
    from voxsrc2020_speaker_verification_amd import kaldi
    from voxsrc2020_speaker_verification_amd.extractor import Extractor
    from voxsrc2020_speaker_verification_amd.stream import extract_entries
    spec, t, blob = weights(name, 80)
    entries = kaldi.read_scp(_cm_ark(tmp_path, LENS * 2, 4))
    exs = [Extractor(blob, device=0, precision="bf16") for _ in range(lanes)]
    try:
        k0, host = extract_entries(entries, exs, batch=6, device_reader=False)
        k1, devr = extract_entries(entries, exs, batch=6, device_reader=True)
        k2, exact = extract_entries(entries, exs, batch=6, device_reader=True, ragged=False)
    finally:
        for e in exs:
            e.close()
    assert k0 == k1 == k2 == [k for k, _ in entries]
    assert np.array_equal(devr.view(np.uint32), host.view(np.uint32))
    assert np.array_equal(exact.view(np.uint32), host.view(np.uint32))
