"""Shared pieces of the SMILES-based examples (reference ``examples/{ogb, zinc, csce,
dftb_uv_spectrum}``): their datasets (PCQM4Mv2 / ZINC / CSCE / DFTB UV spectra) are
CSV or pickled SMILES tables that cannot be downloaded here.

``make_table(n, kind)`` writes the same kind of table from synthetic molecules: SMILES
strings assembled from chemically valid fragments (chains, branches, carbonyls,
nitriles, halogens, para-phenylene / pyridine rings) and targets that are smooth
functions of the structure (so the models have something to learn):

* ``gap``      HOMO-LUMO-gap-like: decreases with conjugation (aromatic rings, double /
               triple bonds), shifted by heteroatoms;
* ``logp``     ZINC's penalised-logP-like: carbons/halogens raise it, N/O lower it;
* ``spectrum`` a UV-like absorption curve on a wavelength grid (Gaussian bands whose
               positions follow the conjugation length);
* ``discrete`` the (peak energies, intensities) pair of the discrete-spectrum config.

Graphs come from the framework's RDKit-free SMILES reader
(``hydragnn_amd.utils.smiles.generate_graphdata_from_smilestr``, the reference's
``smiles_utils.py``), then the low-level API: ``create_dataloaders`` ->
``train_model`` -> ``test``.
"""
import csv
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from hydragnn_amd.utils.smiles import generate_graphdata_from_smilestr, parse_smiles  # noqa: E402

# chain units (left end bonds to the previous unit, right end to the next)
_UNITS = ["C", "C", "CC", "C(C)", "C(=O)", "N", "O", "S", "C(F)(F)", "C=C", "c1ccc(cc1)", "c1cnc(cc1)", "C(Cl)",
          "C#C", "C(O)", "N(C)"]
_CAPS = ["C", "O", "N", "F", "Cl", "C#N", "c1ccccc1", "C(=O)O", "Br"]


def random_smiles(rng, min_units=1, max_units=7):
    n = int(rng.integers(min_units, max_units + 1))
    s = "".join(rng.choice(_UNITS) for _ in range(n)) + str(rng.choice(_CAPS))
    return s.replace("C#CC#C", "C#CCC#C")


def descriptors(smiles):
    m = parse_smiles(smiles)
    sym = [a.symbol for a in m.atoms]
    arom = sum(1 for a in m.atoms if a.aromatic)
    dbl = sum(1 for _, _, o in m.bonds if o == 2.0)
    tri = sum(1 for _, _, o in m.bonds if o == 3.0)
    return dict(n=len(sym), C=sym.count("C"), N=sym.count("N"), O=sym.count("O"),
                hal=sum(sym.count(x) for x in ("F", "Cl", "Br")), S=sym.count("S"), arom=arom, dbl=dbl, tri=tri,
                H=sum(m.num_hs))


def target_gap(d):
    conj = d["arom"] / 6.0 + 0.5 * d["dbl"] + 0.7 * d["tri"]
    return 9.0 - 1.6 * np.log1p(conj) - 0.15 * d["N"] - 0.1 * d["O"] + 0.05 * d["hal"]


def target_logp(d):
    return 0.45 * d["C"] + 0.6 * d["hal"] - 0.8 * d["N"] - 0.7 * d["O"] + 0.3 * d["S"] + 0.2 * d["arom"] / 6 - 1.0


def target_spectrum(d, grid):
    conj = d["arom"] / 6.0 + 0.5 * d["dbl"] + 0.7 * d["tri"]
    bands = [(180.0 + 40.0 * conj, 1.0 + 0.2 * conj), (230.0 + 60.0 * conj, 0.3 + 0.4 * conj),
             (160.0 + 5.0 * d["N"] + 4.0 * d["O"], 0.5)]
    return sum(a * np.exp(-0.5 * ((grid - c) / 12.0) ** 2) for c, a in bands)


def target_discrete(d, npeaks):
    conj = d["arom"] / 6.0 + 0.5 * d["dbl"] + 0.7 * d["tri"]
    e = 6.5 - 0.9 * np.log1p(conj) + 0.4 * np.arange(npeaks)
    f = (0.2 + 0.1 * conj) / (1.0 + np.arange(npeaks))
    return e, f


def make_table(path, n, kind, seed=0, spectrum_dim=500, npeaks=4, elements=None):
    """Write a CSV like the reference datasets: ``smiles,<target columns>``; ``elements``
    restricts the heavy atoms to a dataset's type table."""
    rng = np.random.default_rng(seed)
    grid = np.linspace(150.0, 450.0, spectrum_dim)
    seen, rows = set(), []
    while len(rows) < n:
        s = random_smiles(rng)
        if s in seen and len(seen) < 5000:
            continue
        if elements is not None and any(a.symbol not in elements for a in parse_smiles(s).atoms):
            continue
        seen.add(s)
        d = descriptors(s)
        if kind == "gap":
            y = [target_gap(d)]
        elif kind == "logp":
            y = [target_logp(d)]
        elif kind == "spectrum":
            y = list(target_spectrum(d, grid))
        elif kind == "discrete":
            e, f = target_discrete(d, npeaks)
            y = list(e) + list(f)
        else:
            raise ValueError(kind)
        rows.append([s] + [f"{v:.6g}" for v in y])
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["smiles"] + [f"y{i}" for i in range(len(rows[0]) - 1)])
        w.writerows(rows)
    return path


def read_table(path):
    with open(path) as fh:
        r = csv.reader(fh)
        next(r)
        rows = list(r)
    return [row[0] for row in rows], [np.asarray(row[1:], dtype=np.float32) for row in rows]


def graphs_from_table(smiles, targets, types, var_config):
    out = []
    for s, y in zip(smiles, targets):
        out.append(generate_graphdata_from_smilestr(s, torch.from_numpy(y).view(-1, 1), types, var_config))
    return out


def train_and_test(config, samples, log_name, seed=0):
    """Low-level API path of the reference drivers: split -> create_dataloaders ->
    train_model -> test.  Returns the result dict (also printed as JSON)."""
    import hydragnn_amd
    from hydragnn_amd.data.load_data import create_dataloaders
    from hydragnn_amd.data.splitting import split_dataset
    from hydragnn_amd.parallel.distributed import get_comm_size_and_rank, setup_ddp
    from hydragnn_amd.train.train_validate_test import test

    setup_ddp()
    torch.manual_seed(seed)
    tr, va, te = split_dataset(samples, config["NeuralNetwork"]["Training"].get("perc_train", 0.8), False)
    loaders = create_dataloaders(tr, va, te, config["NeuralNetwork"]["Training"]["batch_size"])
    model = hydragnn_amd.train_model(config, *loaders, log_name=log_name)
    err, tasks, true_v, pred_v = test(loaders[2], model, 0)
    res = {"log_name": log_name, "test_error": float(err), "task_errors": [float(t) for t in tasks],
           "num_train": len(tr)}
    if get_comm_size_and_rank()[1] == 0:
        print(json.dumps(res), flush=True)
    return res


def var_config_for(config, graph_feature_dims, num_node_features):
    v = config["NeuralNetwork"]["Variables_of_interest"]
    v["graph_feature_dims"] = list(graph_feature_dims)
    v["input_node_feature_dims"] = [1] * num_node_features
    v.setdefault("input_node_features", list(range(num_node_features)))
    return v


def parser(desc, default_config):
    import argparse

    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--inputfile", default=default_config)
    ap.add_argument("--csv", default=None, help="existing table (smiles,targets...); generated when absent")
    ap.add_argument("--num_samples", type=int, default=1000)
    ap.add_argument("--num_epoch", type=int, default=None)
    ap.add_argument("--batch_size", type=int, default=None)
    ap.add_argument("--workdir", default=None)
    ap.add_argument("--seed", type=int, default=0)
    return ap


def load(here, args):
    path = args.inputfile if os.path.isabs(args.inputfile) else os.path.join(here, args.inputfile)
    with open(path) as f:
        config = json.load(f)
    tr = config["NeuralNetwork"]["Training"]
    if args.num_epoch is not None:
        tr["num_epoch"] = args.num_epoch
    if args.batch_size is not None:
        tr["batch_size"] = args.batch_size
    workdir = os.path.abspath(args.workdir or os.getcwd())
    os.makedirs(workdir, exist_ok=True)
    os.chdir(workdir)
    return config, workdir
