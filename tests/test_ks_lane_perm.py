"""conv3x3_ks's lane -> pixel table (csrc/conv3k.hip g_ks_perm) is what
tools/ks_lane_perm.py derives, every row is a permutation of the 32 group
pixels, and under the gfx950 ds_read_b128 bank model it reads the window with
fewer LDS cycles than the identity assignment (8 -> 5.625 per read at W = 20)."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import ks_lane_perm  # noqa: E402


def _hip_table():
    src = open(os.path.join(ROOT, "voxsrc2020_speaker_verification_amd", "csrc", "conv3k.hip")).read()
    body = src[src.index("g_ks_perm[2][5][32] = {"):]
    body = body[:body.index("};")]
    rows = [list(map(int, r.split(","))) for r in re.findall(r"\{([\d,\s]+)\}", body)]
    assert len(rows) == 10
    return {20: rows[:5], 10: rows[5:]}


def test_table_matches_generator():
    assert _hip_table() == ks_lane_perm.tables()


def test_rows_are_permutations_and_cut_bank_cycles():
    tab = _hip_table()
    for W, rows in tab.items():
        for r in rows:
            assert sorted(r) == list(range(32))
        base = ks_lane_perm.read_cycles(W, None, tiles=3)
        perm = ks_lane_perm.read_cycles(W, rows, tiles=3)
        assert perm < base - 1.5, (W, base, perm)
