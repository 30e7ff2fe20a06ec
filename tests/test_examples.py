"""Example smoke tests (reference ``tests/test_examples.py``: qm9 / md17 / LennardJones
drivers run as subprocesses).  Tiny sample counts and 1-2 epochs: they check that
each driver's data generation, config and training path run end to end on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")


def _run(script, args, tmp_path, nproc=1, timeout=300, device_data="0"):
    env = dict(os.environ, HYDRAGNN_DEVICE_DATA=device_data, OMP_NUM_THREADS="2")
    if nproc == 1:
        cmd = [sys.executable, os.path.join(EX, script), "--workdir", str(tmp_path)] + args
        env["HYDRAGNN_MASTER_PORT"] = str(29000 + (abs(hash(script + str(args))) % 2000))
    else:
        # torchrun's MASTER_PORT must win: an inherited HYDRAGNN_MASTER_PORT (conftest gives each
        # xdist worker one, and the worker may hold a process group on it) would override it
        env.pop("HYDRAGNN_MASTER_PORT", None)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", f"--master-port={31000 + abs(hash(script)) % 2000}",
               os.path.join(EX, script), "--workdir", str(tmp_path)] + args
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _result(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    return json.loads(lines[-1])


@pytest.mark.parametrize("mpnn_type", ["SchNet", "PNA", "EGNN"])
def test_qm9(mpnn_type, tmp_path):
    r = _result(_run("qm9/qm9.py", ["--num_samples", "40", "--num_epoch", "1", "--mpnn_type", mpnn_type], tmp_path))
    assert r["test_error"] == r["test_error"]  # finite, not NaN


def test_md17_graph_energy(tmp_path):
    r = _result(_run("md17/md17.py", ["--num_samples", "30", "--num_epoch", "1"], tmp_path))
    assert r["test_error"] == r["test_error"]


@pytest.mark.parametrize("mpnn_type", ["PAINN", "SchNet"])
def test_md17_forces(mpnn_type, tmp_path):
    r = _result(_run("md17/md17.py", ["--inputfile", "md17_forces.json", "--num_samples", "24", "--num_epoch", "2",
                                      "--mpnn_type", mpnn_type], tmp_path))
    assert r["test_error"] == r["test_error"]


@pytest.mark.parametrize("mpnn_type", ["PNAPlus", "SchNet", "DimeNet", "EGNN", "PNAEq", "PAINN", "MACE"])
def test_lennard_jones_forces(mpnn_type, tmp_path):
    """Reference ``tests/test_examples.py:65-87``: the LJ grad-forces example over all 7 stacks
    whose energies depend on positions (forces = -dE/dpos, double backward)."""
    r = _result(_run("LennardJones/lj.py", ["--num_samples", "20", "--num_epoch", "2", "--mpnn_type", mpnn_type],
                     tmp_path))
    assert r["test_error"] == r["test_error"]


@pytest.mark.parametrize("cfg", ["open_catalyst_energy.json", "open_catalyst_gps.json"])
def test_open_catalyst(cfg, tmp_path):
    r = _result(_run("open_catalyst_2020/train.py", ["--inputfile", cfg, "--num_samples", "24", "--num_epoch", "1"],
                     tmp_path))
    assert r["test_error"] == r["test_error"]


def test_multibranch_data_parallel(tmp_path):
    r = _result(_run("multibranch/train.py", ["--num_samples", "40", "--num_epoch", "1"], tmp_path))
    assert len(r["task_errors"]) == 2


@pytest.mark.parametrize("device_data", ["0", "2"])
def test_multibranch_task_parallel_three_ranks(tmp_path, device_data):
    """device_data=2: the store + statically padded TrainStep path (the CPU twin of the
    captured step) drives MultiTaskModelMP with its two bucketed gradient syncs."""
    _run("multibranch/train.py", ["--task_parallel", "--num_samples", "40", "--num_epoch", "1"], tmp_path, nproc=3,
         device_data=device_data)
    logs = os.listdir(os.path.join(tmp_path, "logs"))
    assert sum(1 for d in logs if "_branch" in d) == 3


@pytest.mark.slow
def test_lsms(tmp_path):
    r = _result(_run("lsms/lsms.py", ["--num_samples", "300", "--num_epoch", "2"], tmp_path))
    assert len(r["task_errors"]) == 3


@pytest.mark.parametrize("fmt", ["pickle", "columnar"])
def test_ising_model(fmt, tmp_path):
    """Reference ``examples/ising_model``: generated configurations -> raw pipeline ->
    pickle / columnar stores -> train_model."""
    r = _result(_run("ising_model/train_ising.py", ["--histogram_cutoff", "8", "--num_epoch", "1", "--format", fmt],
                     tmp_path))
    assert len(r["task_errors"]) == 2 and r["test_error"] == r["test_error"]


def test_ising_model_ddstore_two_ranks(tmp_path):
    _run("ising_model/train_ising.py", ["--histogram_cutoff", "8", "--num_epoch", "1", "--ddstore"], tmp_path,
         nproc=2)


@pytest.mark.parametrize("cfg,fmt", [("NiNb_EAM_multitask.json", "--pickle"),
                                     ("NiNb_EAM_bulk_multitask.json", "--adios")])
def test_eam(cfg, fmt, tmp_path):
    """Reference ``examples/eam``: EAM CFG files -> CFGDataset -> serialized/columnar store."""
    r = _result(_run("eam/eam.py", ["--inputfile", cfg, "--num_samples", "40", "--num_epoch", "1", fmt], tmp_path))
    assert len(r["task_errors"]) == (2 if "bulk" not in cfg else 3)


def test_multidataset_single_rank(tmp_path):
    r = _result(_run("multidataset/train.py", ["--multi_model_list", "ANI1x", "--prepare_samples", "40",
                                               "--num_epoch", "1"], tmp_path))
    assert r["datasets"] == ["ANI1x"]


def test_multidataset_three_ranks_and_ddstore(tmp_path):
    """Reference ``examples/multidataset --multi``: ranks split over two stores in proportion
    to their sizes, merged PNA histograms; then the same stores through ``--ddstore``."""
    _run("multidataset/train.py", ["--multi_model_list", "ANI1x,QM7-X", "--prepare_samples", "40", "--num_epoch", "1"],
         tmp_path, nproc=3)
    _run("multidataset/train.py", ["--multi_model_list", "ANI1x,QM7-X", "--num_epoch", "1", "--ddstore"], tmp_path,
         nproc=2)


_FAMILIES = ["qm7x", "ani1_x", "transition1x", "open_molecules_2025", "mptrj", "alexandria", "open_materials_2024",
             "open_catalyst_2022", "open_direct_air_capture_2023"]


@pytest.mark.parametrize("family", _FAMILIES)
def test_atomistic_family(family, tmp_path):
    """Every dataset-family driver (examples/atomistic.py) trains EGNN end to end; energy and
    forces configs alternate across the families."""
    task = "forces" if _FAMILIES.index(family) % 2 else "energy"
    n = "12" if family == "open_direct_air_capture_2023" else "30"
    r = _result(_run(f"{family}/train.py", ["--inputfile", f"{family}_{task}.json", "--num_samples", n,
                                             "--num_epoch", "1"], tmp_path))
    assert r["test_error"] == r["test_error"]


@pytest.mark.parametrize("family", ["qm7x", "mptrj", "open_catalyst_2022"])
def test_atomistic_forces_are_gradients(family):
    """The synthetic potential's analytic forces equal -dE/dpos (central differences)."""
    import numpy as np
    import torch

    sys.path.insert(0, EX)
    import atomistic as A

    fam = A.FAMILIES[family]
    rng = np.random.default_rng(3)
    g = A.make_sample(rng, fam)
    pos = g.pos.double().numpy()
    z = g.x[:, 0].long().numpy()
    cell = g.cell.double().numpy() if g.get("cell") is not None else None

    def energy(p):
        if cell is not None:
            ei, sh = A.radius_graph_pbc(torch.from_numpy(p), torch.from_numpy(cell), list(fam.pbc_axes), fam.radius,
                                        max_num_neighbors=10 ** 6)
            src, dst = ei[0].numpy(), ei[1].numpy()
            vec = p[dst] - p[src] + sh.numpy().astype(np.float64)
        else:
            r = np.linalg.norm(p[:, None] - p[None], axis=-1)
            dst, src = np.nonzero((r < fam.radius) & (r > 0))
            vec = p[dst] - p[src]
        return A._energy_forces(z, p, src, dst, vec)

    e0, f0 = energy(pos)
    # recompute f0 in float64 (the sample stores float32)
    for a, k in [(0, 0), (len(pos) // 2, 1), (len(pos) - 1, 2)]:
        h = 1e-5
        pp, pm = pos.copy(), pos.copy()
        pp[a, k] += h
        pm[a, k] -= h
        fd = -(energy(pp)[0] - energy(pm)[0]) / (2 * h)
        assert abs(fd - f0[a, k]) < 1e-4 * max(1.0, abs(fd)), (a, k, fd, f0[a, k])


@pytest.mark.parametrize("script", ["ogb/train_gap.py", "csce/train_gap.py", "zinc/zinc.py",
                                    "dftb_uv_spectrum/train_smooth_uv_spectrum.py",
                                    "dftb_uv_spectrum/train_discrete_uv_spectrum.py"])
def test_smiles_examples(script, tmp_path):
    """SMILES-table examples (RDKit-free reader) train end to end through the low-level API."""
    r = _result(_run(script, ["--num_samples", "48", "--num_epoch", "1"], tmp_path))
    assert r["test_error"] == r["test_error"] and r["num_train"] > 0


def test_qm9_hpo_random_search(tmp_path):
    """examples/qm9_hpo: random search, trials as torchrun children on disjoint slots."""
    out = _run("qm9_hpo/qm9_hpo.py", ["--trials", "2", "--gpus", "2", "--num_epoch", "1", "--num_samples", "40"],
               tmp_path, timeout=600)
    r = _result(out)
    assert r["n_ok"] == 2 and r["best_test_error"] == r["best_test_error"]


def test_multidataset_deepspeed_zero(tmp_path):
    """examples/multidataset_deepspeed --zero_opt: the GFM driver on ZeRO-1, two ranks."""
    out = _run("multidataset_deepspeed/train.py", ["--zero_opt", "--num_epoch", "1", "--num_samples", "24",
                                                   "--prepare_samples", "50"], tmp_path, nproc=2, timeout=600)
    r = _result(out)
    assert r["test_error"] == r["test_error"]
    cfg = json.load(open(os.path.join(str(tmp_path), "deepspeed_derived_config_rank0.json")))
    assert cfg["NeuralNetwork"]["Training"]["Optimizer"]["use_zero_redundancy"] is True


def test_multidataset_inference_reproduces_test_error(tmp_path):
    """examples/multidataset/inference.py on a freshly trained GFM log: same test error as training."""
    tr = _result(_run("multidataset/train.py", ["--adios", "--modelname", "ANI1x", "--num_epoch", "1",
                                                "--num_samples", "30", "--prepare_samples", "60"], tmp_path))
    out = _run("multidataset/inference.py", ["--log", "GFM", "--datasets", "ANI1x"], tmp_path)
    inf = _result(out)
    assert abs(inf["test_error"] - tr["test_error"]) < 1e-5 * max(1.0, tr["test_error"])
    assert inf["graphs_per_s"] > 0


def test_multibranch_task_parallel_device_mesh(tmp_path):
    """--use_devicemesh: branch groups from a 2-D device mesh (2 branches x 2 replicas)."""
    _run("multibranch/train.py", ["--task_parallel", "--use_devicemesh", "--num_datasets", "2", "--num_samples", "40",
                                  "--num_epoch", "1"], tmp_path, nproc=4)
    logs = os.listdir(os.path.join(tmp_path, "logs"))
    assert sum(1 for d in logs if "_branch" in d) == 2
