"""Multi-dataset, multi-branch foundation-model training (reference
``examples/multibranch/train.py`` + ``multibranch_GFM260_SC25.json``).

Every dataset k is routed to decoder branch ``branch-k`` through
``data.dataset_name``; the heads are a graph energy head and a node force head
(task weights [1, 100]).  Two parallel modes (reference ``--task_parallel``):

* data parallel (default): every rank sees all datasets, one world-wide DDP;
* task parallel (``--task_parallel``): ranks are split over datasets in
  proportion to their sizes (``models.multitask.branch_groups``), each rank
  reads only its dataset, and ``MultiTaskModelMP`` syncs the shared encoder
  over the world and each branch decoder over its branch group (branches of
  other datasets are pruned from the rank's model).

``--nosync`` disables gradient synchronisation for the whole run (reference
``--nosync``), ``--oversampling`` uses random oversampling to
``--oversampling_num_samples`` per epoch.  Configs: ``multibranch_GFM.json``
(3 branches, EGNN hidden 128 — CI size) and ``multibranch_GFM260_SC25.json``
(the SC25 shape: EGNN hidden 866 x 4 layers, 5 branches, heads 3 x 889).

The five SC25 datasets (ANI1x, QM7-X, MPTrj, Alexandria, Transition1x) are not
downloadable here: each branch gets its own synthetic family (molecules of
different sizes / element mixes, or OC20-like condensed systems), with energies
and exact forces of a smooth pseudo-potential.

Usage: python examples/multibranch/train.py [--num_datasets 3] [--task_parallel]
       torchrun --nproc-per-node 4 examples/multibranch/train.py --task_parallel
"""
import contextlib
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from common import base_parser, load_config, run_example, split  # noqa: E402

from hydragnn_amd.data.graph import Graph  # noqa: E402
from hydragnn_amd.data.synthetic import molecules_like  # noqa: E402


def family(k, num, seed):
    """Synthetic dataset k: molecules whose size range grows with k."""
    lo, hi = 4 + 3 * k, 12 + 6 * k
    out = []
    for s in molecules_like(num, seed=seed + 1000 * k, min_atoms=lo, max_atoms=hi, with_forces=True):
        x = torch.cat([s.x, s.pos, s.forces], 1)  # atomic_number | cartesian coordinates | forces
        out.append(Graph(x=x, pos=s.pos, y=s.y, energy=s.energy, forces=s.forces,
                         dataset_name=torch.tensor([[k]], dtype=torch.int64)))
    return out


def _task_parallel(config, datasets, args):
    import torch.distributed as dist

    from hydragnn_amd.data.load_data import create_dataloaders
    from hydragnn_amd.data.serialized import SerializedDataLoader
    from hydragnn_amd.models.create import create_model_config
    from hydragnn_amd.models.multitask import MultiTaskModelMP, branch_groups
    from hydragnn_amd.parallel.distributed import setup_ddp
    from hydragnn_amd.train.train_validate_test import train_validate_test
    from hydragnn_amd.utils.config_utils import get_log_name_config, save_config, update_config
    from hydragnn_amd.utils.model import get_summary_writer, save_model
    from hydragnn_amd.utils.optimizer import select_optimizer
    from hydragnn_amd.utils.print_utils import setup_log

    setup_ddp()
    if args.use_devicemesh:
        from hydragnn_amd.models.multitask import branch_groups_mesh

        bid, group, lists = branch_groups_mesh(len(datasets))
    else:
        bid, group, lists = branch_groups([len(d) for d in datasets])
    mine = datasets[bid]
    tr, va, te = split(mine, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    proc = SerializedDataLoader(config)
    tr, va, te = proc.process(tr), proc.process(va), proc.process(te)
    bs = config["NeuralNetwork"]["Training"]["batch_size"]
    tl, vl, tel = create_dataloaders(tr, va, te, bs, group=group)
    config = update_config(config, tl, vl, tel)
    log_name = get_log_name_config(config) + f"_tp{dist.get_world_size()}"
    setup_log(log_name)
    base = create_model_config(config["NeuralNetwork"], verbosity=config["Verbosity"]["level"])
    model = MultiTaskModelMP(base, bid, group)
    opt = select_optimizer(model, config["NeuralNetwork"]["Training"]["Optimizer"])
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=5, min_lr=1e-5)
    if dist.get_rank() == 0:
        save_config(config, log_name)
    engine = None
    if not args.nosync:
        # GPU: HBM-resident branch shard + captured step with both gradient syncs in the graph
        from hydragnn_amd.run_training import make_step_engine

        engine, (tl, vl, tel) = make_step_engine(config, model, opt, (tl, vl, tel))
    ctx = model.no_sync() if args.nosync else contextlib.nullcontext()
    with ctx:
        train_validate_test(model, opt, tl, vl, tel, get_summary_writer(log_name), sched, config["NeuralNetwork"],
                            log_name, config["Verbosity"]["level"],
                            compute_grad_energy=config["NeuralNetwork"]["Training"].get("compute_grad_energy", False),
                            step_engine=engine)
    save_model(model, opt, log_name)  # -> <log_name>_branch<B>.pk, rank 0 of every branch group
    return {"branch": bid, "ranks": lists}


def main(argv=None):
    ap = base_parser(__doc__.splitlines()[0], "multibranch_GFM.json")
    ap.add_argument("--num_datasets", type=int, default=None, help="default: number of branches in the config")
    ap.add_argument("--task_parallel", action="store_true")
    ap.add_argument("--nosync", action="store_true")
    ap.add_argument("--use_devicemesh", action="store_true",
                    help="task parallel: branch groups from a 2-D device mesh (equal rank split)")
    ap.add_argument("--oversampling", action="store_true")
    ap.add_argument("--oversampling_num_samples", type=int, default=None)
    args = ap.parse_args(argv)
    config = load_config(HERE, args)
    nb = len(config["NeuralNetwork"]["Architecture"]["output_heads"]["graph"])
    K = args.num_datasets or nb
    assert K <= nb, f"{K} datasets but only {nb} branches in the config"
    n = args.num_samples or 200
    datasets = [family(k, max(8, n // (k + 1)), args.seed) for k in range(K)]  # unequal sizes
    if args.task_parallel:
        return _task_parallel(config, datasets, args)
    allsamples = [s for d in datasets for s in d]
    tr, va, te = split(allsamples, config["NeuralNetwork"]["Training"]["perc_train"], seed=args.seed)
    return run_example(config, tr, va, te, args.workdir)


if __name__ == "__main__":
    main()
