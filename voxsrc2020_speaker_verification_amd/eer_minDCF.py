"""CLI mirror of tensorflow/eer_minDCF.py:67-94 (same flags and printout)."""

import argparse
import sys

from .scoring import eer_from_files


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--c-miss", type=float, dest="c_miss", default=1)
    ap.add_argument("--c-fa", type=float, dest="c_fa", default=1)
    ap.add_argument("--p-target", type=float, dest="p_target", default=0.01)
    ap.add_argument("--trial", type=str)
    ap.add_argument("--score", type=str)
    a = ap.parse_args(argv)
    eer, thr, mindcf, mthr = eer_from_files(a.trial, a.score, a.c_miss, a.c_fa, a.p_target)
    print("EER is {:.4f}%, at threshold: {:.4f}".format(eer * 100, thr))
    print("minDCF is {:.4f}, at threshold: {:.4f} (p-target={}, c-miss={}, c-fa={})".format(
        mindcf, mthr, a.p_target, a.c_miss, a.c_fa))
    return 0


if __name__ == "__main__":
    sys.exit(main())
