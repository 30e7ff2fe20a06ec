"""Hyper-parameter search on the multi-dataset GFM driver (reference
``examples/multidataset_hpo/{gfm.py, gfm_deephyper_multi.py}``: DeepHyper over model type,
width, depth and learning rate, each trial a multi-GPU ``gfm.py`` run on the merged
ANI1x / QM7-X / MPTrj / ... stores).

Random search (``hydragnn_amd.utils.hpo``) over the same space; every trial is
``examples/multidataset/train.py`` launched with ``torchrun`` on its own GPU slot
(``--gpus_per_trial`` ranks each, so a trial exercises the per-dataset process groups
and the proportional rank assignment of the GFM driver).

Usage: python examples/multidataset_hpo/gfm_hpo.py [--trials 4] [--gpus 8] [--gpus_per_trial 2]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "examples", "qm9_hpo"))
from qm9_hpo import search  # noqa: E402

SPACE = {
    "--mpnn_type": ["EGNN", "SchNet", "PNAPlus", "PAINN"],
    "--hidden_dim": ["32", "50", "64"],
    "--num_conv_layers": ["2", "3"],
    "--learning_rate": ["0.0005", "0.001", "0.002"],
}

if __name__ == "__main__":
    argv = sys.argv[1:]
    if "--num_samples" not in argv:
        argv += ["--num_samples", "100"]
    if "--gpus_per_trial" not in argv:  # --multi needs a rank per dataset (ANI1x, QM7-X)
        argv += ["--gpus_per_trial", "2"]
    search(os.path.join(ROOT, "examples", "multidataset", "train.py"), SPACE, argv + ["--prepare_samples", "120"],
           __doc__.splitlines()[0])
