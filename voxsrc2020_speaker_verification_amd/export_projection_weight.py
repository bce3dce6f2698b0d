"""CLI mirror of tensorflow/export_projection_weight.py: the margin head's
weight variable -> the l2-normalised projection matrix snorm.py takes as its
`--weight_matrix` cohort (one row per class centre).

The reference reads the variable from a TF checkpoint
(`tf.train.NewCheckpointReader`, export_projection_weight.py:28-31) and
pickles the result (:47).  TensorFlow is not part of this build and pickles
are not loaded, so the variable comes in as a `.npy` array (e.g. written by
`pb2blob`-style tooling from the checkpoint) and the matrix goes out as `.npy`;
the arithmetic between the two is the reference's (:32-35):
swapaxes(-1, -2) -> reshape(-1, last) -> row l2norm.

    python -m voxsrc2020_speaker_verification_amd.export_projection_weight \\
        --input_npy head_kernel.npy --output_weight proj.npy
"""

import argparse
import sys

import numpy as np

from .scoring import l2norm


def projection_weight(var):
    """export_projection_weight.py:28-35 (after the checkpoint read)."""
    weight = np.swapaxes(np.asarray(var), -1, -2)
    weight = np.reshape(weight, (-1, weight.shape[-1]))
    return l2norm(weight, axis=1)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input_npy", type=str, required=True,
                    help="the head's weight variable as .npy (the reference reads a TF checkpoint)")
    ap.add_argument("--output_weight", type=str, required=True, help="output .npy matrix")
    a = ap.parse_args(argv)
    np.save(a.output_weight, projection_weight(np.load(a.input_npy, allow_pickle=False)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
