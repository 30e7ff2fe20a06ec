"""Auxiliary utilities: LSMS formation enthalpy (reference ``tests/test_enthalpy.py``),
compositional histogram cutoff, atomic descriptors (reference
``tests/test_atomicdescriptors.py`` runs the script; here the computed layout is
checked), and the HPO trial scheduler (2 concurrent CPU trials of the qm9 example)."""
import json
import os
import sys

import numpy as np
import pytest
import torch

from hydragnn_amd.data.lsms import deterministic_graph_data
from hydragnn_amd.utils.lsms import compositional_histogram_cutoff, convert_raw_data_energy_to_gibbs


def test_formation_enthalpy(tmp_path):
    d = str(tmp_path / "unit_test_enthalpy")
    deterministic_graph_data(d, number_configurations=10, number_types=2, linear_only=True, seed=1)
    deterministic_graph_data(d, number_configurations=1, configuration_start=10, number_types=1, types=[0],
                             linear_only=True, seed=2)
    deterministic_graph_data(d, number_configurations=1, configuration_start=11, number_types=1, types=[1],
                             linear_only=True, seed=3)
    convert_raw_data_energy_to_gibbs(d, [0, 1], create_plots=False)
    new = d + "_gibbs_energy"
    files = os.listdir(new)
    assert len(files) == 12
    for fn in files:  # linear-only energies: zero formation enthalpy
        assert abs(float(np.loadtxt(os.path.join(new, fn), max_rows=1).reshape(-1)[0])) < 1e-6


def test_compositional_histogram_cutoff(tmp_path):
    d = str(tmp_path / "raw")
    deterministic_graph_data(d, number_configurations=40, number_types=2, seed=4)
    comp, allc = compositional_histogram_cutoff(d, [0, 1], histogram_cutoff=3, num_bins=5)
    assert len(os.listdir(d + "_histogram_cutoff")) == len(comp) <= 2 * 5
    assert allc.sum() == 40


def test_atomic_descriptors(tmp_path):
    from hydragnn_amd.utils.descriptors import atomicdescriptors, group_block_of, valence_electrons

    assert group_block_of(6) == (14, 1) and group_block_of(26) == (8, 2) and group_block_of(79) == (11, 2)
    assert group_block_of(64)[1] == 3 and group_block_of(86) == (18, 1) and group_block_of(1) == (1, 0)
    assert valence_electrons(8) == 6 and valence_electrons(11) == 1 and valence_electrons(29) == 11
    a = atomicdescriptors(str(tmp_path / "emb.json"), element_types=["C", "H", "O", "N", "F", "S"])
    assert sorted(int(k) for k in a.atom_embeddings) == [1, 6, 7, 8, 9, 16]
    f = a.get_atom_features(8)
    # [type_id, group, period, block x4, valence, Z, weight, EN, rcov, IE, has_table]
    assert f[1] == 16 and f[2] == 2 and f[4] == 1 and f[7] == 6 and f[8] == 8  # p block, 6 valence e-
    assert abs(float(f[9]) - 15.999) < 1e-3 and abs(float(f[10]) - 3.44) < 1e-6
    b = atomicdescriptors(str(tmp_path / "emb1.json"), element_types=None, one_hot=True)
    assert len(b.atom_embeddings) == 118
    assert len({len(v) for v in b.atom_embeddings.values()}) == 1


def test_hpo_scheduler_two_slots(tmp_path):
    from hydragnn_amd.utils.hpo import TrialScheduler, random_search

    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "qm9", "qm9.py")
    sched = TrialScheduler(script, total_gpus=2, gpus_per_trial=1, base_port=29950, workdir=str(tmp_path),
                           env={"HYDRAGNN_DEVICE_DATA": "0", "OMP_NUM_THREADS": "2"}, timeout=300)
    best, val, res = random_search({"--mpnn_type": ["SchNet", "GIN"], "--batch_size": ["16", "32"]}, 2, sched,
                                   fixed_args=["--num_samples", "30", "--num_epoch", "1"])
    assert all(r["returncode"] == 0 for r in res), [open(r["log"]).read()[-2000:] for r in res]
    assert best is not None and val == val


def test_loader_threads_affinity_and_custom_flag(monkeypatch):
    """HYDRAGNN_NUM_WORKERS collate threads keep the batch order; HYDRAGNN_AFFINITY pins
    each worker thread to its core window (reference HydraDataLoader.worker_init)."""
    import os
    import threading

    from hydragnn_amd.data import loader as L
    from hydragnn_amd.data.synthetic import oc20_like

    samples = oc20_like(10, seed=1, pe_dim=2, min_atoms=4, max_atoms=8)
    ref = [b.num_graphs for b in L.GraphDataLoader(samples, 3, shuffle=False, num_workers=0)]
    got = [b.num_graphs for b in L.GraphDataLoader(samples, 3, shuffle=False, num_workers=3)]
    assert got == ref
    monkeypatch.setenv("HYDRAGNN_CUSTOM_DATALOADER", "1")
    assert [b.num_graphs for b in L.GraphDataLoader(samples, 3, shuffle=False, num_workers=0)] == ref
    assert L.parse_omp_places("{0:2},{4:2}") == [0, 1, 4, 5] and L.parse_omp_places("{1,3},{7}") == [1, 3, 7]
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) >= 2:
        monkeypatch.setenv("HYDRAGNN_AFFINITY", "1")
        monkeypatch.setenv("HYDRAGNN_AFFINITY_WIDTH", "1")
        out = {}

        def run():
            out["mask"] = L.apply_worker_affinity(1)
            out["now"] = os.sched_getaffinity(0)

        t = threading.Thread(target=run)
        t.start()
        t.join()
        assert out["mask"] == {allowed[1]} and out["now"] == {allowed[1]}
        assert sorted(os.sched_getaffinity(0)) == allowed  # the main thread is untouched


def test_ddstore_epoch_hooks(monkeypatch):
    """HYDRAGNN_USE_ddstore=1 brackets train/validate/test passes with the store's
    epoch_begin / epoch_end (reference train_validate_test.py:468-472)."""
    from hydragnn_amd.train.train_validate_test import _ddstore_epochs

    calls = []

    class DS:
        def epoch_begin(self):
            calls.append("b")

        def epoch_end(self):
            calls.append("e")

    class Loader:
        dataset = DS()

    f = _ddstore_epochs(lambda loader, x: calls.append(x) or x)
    assert f(Loader(), 1) == 1 and calls == [1]
    monkeypatch.setenv("HYDRAGNN_USE_ddstore", "1")
    assert f(Loader(), 2) == 2 and calls == [1, "b", 2, "e"]
