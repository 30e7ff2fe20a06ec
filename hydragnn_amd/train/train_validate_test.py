"""Epoch loop, train / validate / test (reference ``hydragnn/train/train_validate_test.py:39-748``).

Same control flow and outputs as the reference (per-epoch train/val/test losses
and per-task losses, ReduceLROnPlateau on the validation loss, EarlyStopping,
Checkpoint, Slurm walltime guard, ``HYDRAGNN_MAX_NUM_BATCH``,
``HYDRAGNN_VALTEST``, ``HYDRAGNN_TRACE_LEVEL`` region tracing, the profiler
schedule, ``test()`` returning gathered true/predicted values per head).

MI355X data path: when the loaders are ``DeviceGraphLoader`` (HBM-resident
splits) the training batches run through ``TrainStep`` — batch assembly,
forward, backward, gradient all-reduce and the fused optimizer captured as
hipGraphs — and evaluation runs on device-assembled batches.  Host loaders
(``GraphDataLoader``, e.g. CPU/gloo runs) take the eager path.
"""
import os
import time

import torch
import torch.distributed as dist

from ..data.graph import head_targets
from ..data.loader import DeviceGraphLoader
from ..ops.pna import composite_mode
from ..parallel.distributed import check_remaining, get_comm_size_and_rank, get_device
from ..utils import tracer as tr
from ..utils.model import Checkpoint, EarlyStopping
from ..utils.print_utils import iterate_tqdm, print_distributed
from ..utils.profile import Profiler
from ..utils.time_utils import Timer
from .step import TrainStep, batch_loss


def _module(model):
    return model.module if hasattr(model, "module") else model


def get_nbatch(loader, synchronize=False):
    """Batches per epoch (``train_validate_test.py:39-49``).  With ``synchronize`` the count is
    the minimum over ranks: every training batch runs gradient collectives, so ranks whose
    loaders differ in length (task-parallel branches over datasets of different sizes)
    must stop together or their collective sequences diverge."""
    nbatch = len(loader)
    env = os.getenv("HYDRAGNN_MAX_NUM_BATCH")
    if env is not None:
        nbatch = min(nbatch, int(env))
    if synchronize and dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        from ..parallel.distributed import host_group

        t = torch.tensor([nbatch], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=host_group())
        nbatch = int(t.item())
    return nbatch


def prepare_batch(data, module, device):
    """Host batch -> device + per-head targets; device batches pass through."""
    if data.get("targets") is not None:
        return data
    if data.x is not None and data.x.device != device:
        data = data.to(device, non_blocking=True)
    data["targets"] = head_targets(data, module.head_type, module.head_dims) \
        if data.get("y") is not None and data.get("y_loc") is not None else []
    return data


def _loss(module, pred, data, compute_grad_energy):
    if compute_grad_energy:
        return module.energy_force_loss(pred, data)
    return batch_loss(module, pred, data)


@torch.no_grad()
def reduce_values_ranks(local_tensor):
    """Rank average of an error metric; ``HYDRAGNN_AGGR_BACKEND=mpi`` reduces on the host
    (gloo host group, reference ``reduce_values_ranks_mpi``), any value other than
    torch / mpi keeps the rank-local metric."""
    backend = os.getenv("HYDRAGNN_AGGR_BACKEND", "torch")
    if backend not in ("torch", "mpi"):
        return local_tensor
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = local_tensor.clone()
        if backend == "mpi":
            from ..parallel.distributed import host_group

            h = t.detach().cpu()
            dist.all_reduce(h, op=dist.ReduceOp.SUM, group=host_group())
            return h.to(local_tensor.device) / dist.get_world_size()
        if not t.is_cuda and dist.get_backend() != "gloo":
            from ..parallel.distributed import host_group

            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=host_group())
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t / dist.get_world_size()
    return local_tensor


reduce_values_ranks_dist = reduce_values_ranks


@torch.no_grad()
def gather_tensor_ranks(head_values):
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return head_values
    W = dist.get_world_size()
    dev = head_values.device
    size_local = torch.tensor([head_values.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.ones_like(size_local) for _ in range(W)]
    dist.all_gather(sizes, size_local)
    sizes = torch.cat(sizes)
    mx = int(sizes.max())
    padded = torch.zeros((mx,) + tuple(head_values.shape[1:]), dtype=head_values.dtype, device=dev)
    padded[: head_values.shape[0]] = head_values
    lst = [torch.empty_like(padded) for _ in range(W)]
    dist.all_gather(lst, padded)
    return torch.cat([t[: int(s)] for t, s in zip(lst, sizes)], 0)


def _sync_running_stats(model):
    """Broadcast rank 0's BatchNorm running statistics (and any other buffers) once per
    epoch.  torch DDP (the reference's wrapper) broadcasts buffers before every forward;
    the captured step keeps them rank-local inside the step graph, so without this the
    ranks' eval-mode statistics would drift apart.  One collective per buffer per epoch."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    if hasattr(model, "head_pg"):  # MultiTaskModelMP: decoder buffers are branch-local
        return
    module = _module(model)
    with torch.no_grad():
        for b in module.buffers():
            if b.is_floating_point():
                dist.broadcast(b, src=0)


def _ddstore_epochs(fn):
    """``HYDRAGNN_USE_ddstore=1``: bracket the pass over a DistDataset-backed loader with the
    store's ``epoch_begin`` / ``epoch_end`` (reference ``train_validate_test.py:468-472,
    577-581, 634-638``)."""
    import functools

    @functools.wraps(fn)
    def wrapped(loader, *a, **kw):
        ds = getattr(loader, "dataset", None)
        use = bool(int(os.getenv("HYDRAGNN_USE_ddstore", "0"))) and hasattr(ds, "epoch_begin")
        if use:
            ds.epoch_begin()
        try:
            return fn(loader, *a, **kw)
        finally:
            if use:
                ds.epoch_end()

    return wrapped


@_ddstore_epochs
def train(loader, model, opt, verbosity, profiler=None, use_deepspeed=False, compute_grad_energy=False,
          step_engine=None):
    module = _module(model)
    device = next(module.parameters()).device
    total_error = torch.tensor(0.0, device=device)
    tasks_error = torch.zeros(module.num_heads, device=device)
    num_samples = 0
    model.train()
    nbatch = get_nbatch(loader, synchronize=True)
    trace_level = int(os.getenv("HYDRAGNN_TRACE_LEVEL", "0"))
    sync = {"cudasync": trace_level > 0}
    use_engine = step_engine is not None and isinstance(loader, DeviceGraphLoader) and \
        (not compute_grad_energy or getattr(step_engine, "forces", False))
    tr.start("dataload", **sync)
    it = loader.index_batches() if use_engine else iter(loader)
    for ibatch, data in iterate_tqdm(enumerate(it), verbosity, desc="Train", total=nbatch):
        if ibatch >= nbatch:
            break
        tr.stop("dataload", **sync)
        if use_engine:
            tr.start("step", **sync)
            loss, tasks = step_engine(loader.store, data)
            tr.stop("step", **sync)
            ng = len(data)
        else:
            tr.start("zero_grad")
            if step_engine is not None:
                step_engine._zero()
            else:
                opt.zero_grad()
            tr.stop("zero_grad")
            tr.start("forward", **sync)
            data = prepare_batch(data, module, device)
            if compute_grad_energy:
                data.pos.requires_grad_(True)
                with composite_mode(True):
                    pred = model(data)
                    loss, tasks = _loss(module, pred, data, True)
            else:
                pred = model(data)
                loss, tasks = _loss(module, pred, data, False)
            tr.stop("forward", **sync)
            tr.start("backward", **sync)
            if compute_grad_energy:
                with composite_mode(True):
                    loss.backward()
            else:
                loss.backward()
            tr.stop("backward", **sync)
            tr.start("opt_step", **sync)
            if hasattr(opt, "guard"):
                opt.guard = loss.detach()
            opt.step()
            tr.stop("opt_step", **sync)
            ng = data.get("num_graphs_real", data.num_graphs)
        if profiler is not None:
            profiler.step()
        with torch.no_grad():
            total_error += loss.detach() * ng
            num_samples += ng
            for k in range(len(tasks)):
                tasks_error[k] += tasks[k].detach() * ng
        if ibatch < nbatch - 1:
            tr.start("dataload", **sync)
    n = max(num_samples, 1)
    return total_error / n, tasks_error / n


def _eval_batches(loader, nbatch):
    for ibatch, data in enumerate(loader):
        if ibatch >= nbatch:
            break
        yield data


@torch.no_grad()
@_ddstore_epochs
def validate(loader, model, verbosity, reduce_ranks=True, compute_grad_energy=False):
    module = _module(model)
    device = next(module.parameters()).device
    total_error = torch.tensor(0.0, device=device)
    tasks_error = torch.zeros(module.num_heads, device=device)
    num_samples = 0
    model.eval()
    nbatch = get_nbatch(loader)
    for data in iterate_tqdm(_eval_batches(loader, nbatch), verbosity, desc="Validate", total=nbatch):
        data = prepare_batch(data, module, device)
        if compute_grad_energy:
            with torch.enable_grad(), composite_mode(True):
                data.pos.requires_grad_(True)
                pred = model(data)
                err, tasks = _loss(module, pred, data, True)
        else:
            pred = model(data)
            err, tasks = _loss(module, pred, data, False)
        ng = data.get("num_graphs_real", data.num_graphs)
        total_error += err.detach() * ng
        num_samples += ng
        for k in range(len(tasks)):
            tasks_error[k] += tasks[k].detach() * ng
    n = max(num_samples, 1)
    val_error, tasks_error = total_error / n, tasks_error / n
    if reduce_ranks:
        val_error = reduce_values_ranks(val_error)
        tasks_error = reduce_values_ranks(tasks_error)
    return val_error, tasks_error


def _dump_force_samples(records, data, e_pred, e_true, f_pred, f_true):
    """Per-sample energy/force records of ``HYDRAGNN_DUMP_TESTDATA=1`` (reference
    ``train_validate_test.py:642-705``: energy true/pred, flattened forces true/pred, mean
    per-atom force error)."""
    ptr = data.ptr.tolist()
    for i in range(len(ptr) - 1):
        lo, hi = ptr[i], ptr[i + 1]
        ft, fp = f_true[lo:hi].detach().cpu(), f_pred[lo:hi].detach().cpu()
        records.append({"energy_true": float(e_true[i]), "forces_true": ft.flatten(),
                        "energy_pred": float(e_pred[i]), "forces_pred": fp.flatten(),
                        "forces_average_error_per_atom": (ft - fp).norm(dim=1).mean()})


def _dump_samples(records, data, pred, module):
    p = pred[0] if module.var_output else pred
    ptr = data.ptr.tolist()
    for i in range(len(ptr) - 1):
        rec = {}
        for ih in range(module.num_heads):
            t = data.targets[ih]
            if module.head_type[ih] == "graph":
                rec[f"head{ih}_true"], rec[f"head{ih}_pred"] = t[i].detach().cpu(), p[ih][i].detach().cpu()
            else:
                lo, hi = ptr[i], ptr[i + 1]
                rec[f"head{ih}_true"], rec[f"head{ih}_pred"] = t[lo:hi].detach().cpu(), p[ih][lo:hi].detach().cpu()
        records.append(rec)


@torch.no_grad()
@_ddstore_epochs
def test(loader, model, verbosity, reduce_ranks=True, return_samples=True, compute_grad_energy=False):
    """Test-set error (+ per-head true/pred samples).

    Force runs (``compute_grad_energy``) return per-graph energies as head 0's samples
    (prediction = sum of the node-energy head; the round-1 code returned nothing).  With
    ``HYDRAGNN_DUMP_TESTDATA=1`` every rank writes its per-sample records to
    ``testdata_rank{r}.pt`` (a list of dicts of tensors/floats; ``torch.load(...,
    weights_only=True)`` reads it back; the reference pickles the same fields)."""
    module = _module(model)
    device = next(module.parameters()).device
    total_error = torch.tensor(0.0, device=device)
    tasks_error = torch.zeros(module.num_heads, device=device)
    num_samples = 0
    model.eval()
    nbatch = get_nbatch(loader)
    dump = int(os.getenv("HYDRAGNN_DUMP_TESTDATA", "0")) == 1
    records = [] if dump else None
    true_values = [[] for _ in range(module.num_heads)]
    predicted_values = [[] for _ in range(module.num_heads)]
    for data in iterate_tqdm(_eval_batches(loader, nbatch), verbosity, desc="Test", total=nbatch):
        data = prepare_batch(data, module, device)
        if compute_grad_energy:
            with torch.enable_grad(), composite_mode(True):
                data.pos.requires_grad_(True)
                pred = model(data)
                err, tasks = _loss(module, pred, data, True)
                if return_samples or dump:
                    e_pred, e_true, f_pred, f_true = module.energy_force_predict(pred, data, create_graph=False)
            if return_samples:
                true_values[0].append(e_true.detach().reshape(-1, 1))
                predicted_values[0].append(e_pred.detach().reshape(-1, 1))
            if dump:
                _dump_force_samples(records, data, e_pred, e_true, f_pred, f_true)
        else:
            pred = model(data)
            err, tasks = _loss(module, pred, data, False)
            if return_samples:
                p = pred[0] if module.var_output else pred
                for ih in range(module.num_heads):
                    true_values[ih].append(data.targets[ih].reshape(-1, 1))
                    predicted_values[ih].append(p[ih].reshape(-1, 1))
            if dump:
                _dump_samples(records, data, pred, module)
        ng = data.get("num_graphs_real", data.num_graphs)
        total_error += err.detach() * ng
        num_samples += ng
        for k in range(len(tasks)):
            tasks_error[k] += tasks[k].detach() * ng
    if dump:
        from ..parallel.distributed import get_comm_size_and_rank

        torch.save(records, f"testdata_rank{get_comm_size_and_rank()[1]}.pt")
    n = max(num_samples, 1)
    test_error, tasks_error = total_error / n, tasks_error / n
    if return_samples and len(true_values[0]) > 0:
        for ih in range(module.num_heads):
            if true_values[ih]:
                true_values[ih] = torch.cat(true_values[ih], 0)
                predicted_values[ih] = torch.cat(predicted_values[ih], 0)
    if reduce_ranks:
        test_error = reduce_values_ranks(test_error)
        tasks_error = reduce_values_ranks(tasks_error)
        if return_samples and len(true_values[0]) > 0:
            for ih in range(module.num_heads):
                true_values[ih] = gather_tensor_ranks(true_values[ih])
                predicted_values[ih] = gather_tensor_ranks(predicted_values[ih])
    return test_error, tasks_error, true_values, predicted_values


def _record_trainer_state(st, epoch, scheduler, earlystopper, checkpoint):
    st["epoch"] = epoch + 1
    if scheduler is not None and hasattr(scheduler, "state_dict"):
        st["scheduler"] = {k: v for k, v in scheduler.state_dict().items() if isinstance(v, (int, float, str, list))}
    if earlystopper is not None:
        st["early_stopping"] = earlystopper.state_dict()
    if checkpoint is not None:
        st["checkpoint_min"] = float(checkpoint.min_perf_metric)
    st["torch_rng"] = torch.get_rng_state()
    if torch.cuda.is_available():
        st["cuda_rng"] = torch.cuda.get_rng_state_all()


def restore_trainer_state(st, scheduler=None):
    """Scheduler + RNG part of a loaded trainer state (epoch / early stop / checkpoint
    counters are applied by ``train_validate_test``)."""
    if st is None:
        return
    if scheduler is not None and "scheduler" in st:
        sd = scheduler.state_dict()
        sd.update(st["scheduler"])
        scheduler.load_state_dict(sd)
    if "torch_rng" in st:
        torch.set_rng_state(st["torch_rng"])
    if "cuda_rng" in st and torch.cuda.is_available() and len(st["cuda_rng"]) == torch.cuda.device_count():
        torch.cuda.set_rng_state_all(st["cuda_rng"])


def train_validate_test(model, optimizer, train_loader, val_loader, test_loader, writer, scheduler, config,
                        model_with_config_name, verbosity=0, plot_init_solution=True, plot_hist_solution=False,
                        create_plots=False, use_deepspeed=False, compute_grad_energy=False, step_engine=None,
                        trainer_state=None):
    module = _module(model)
    tcfg = config["Training"]
    num_epoch = tcfg["num_epoch"]
    early = tcfg.get("EarlyStopping", False)
    check_time = tcfg.get("CheckRemainingTime", False)
    save_ckpt = tcfg.get("Checkpoint", False)
    device = next(module.parameters()).device
    H = module.num_heads
    total_loss = {k: torch.zeros(num_epoch, device=device) for k in ("train", "val", "test")}
    task_loss = {k: torch.zeros((num_epoch, H), device=device) for k in ("train", "val", "test")}
    visualizer = None
    if create_plots:
        from ..postprocess.visualizer import Visualizer

        node_feature, nodes_num = [], []
        for d in test_loader.dataset:
            node_feature.extend(d.x.tolist())
            nodes_num.append(d.num_nodes)
        visualizer = Visualizer(model_with_config_name, node_feature=node_feature, num_heads=H,
                                head_dims=module.head_dims, num_nodes_list=nodes_num)
        visualizer.num_nodes_plot()
        if plot_init_solution:
            _, _, tv, pv = test(test_loader, model, verbosity)
            visualizer.create_scatter_plots(tv, pv, output_names=config["Variables_of_interest"]["output_names"],
                                            iepoch=-1)
    profiler = Profiler("./logs/" + model_with_config_name)
    if "Profile" in config:
        profiler.setup(config["Profile"])
    earlystopper = EarlyStopping(patience=tcfg.get("patience", 10)) if early else None
    checkpoint = Checkpoint(name=model_with_config_name, warmup=tcfg.get("checkpoint_warmup", 0)) if save_ckpt else None
    if trainer_state is not None:
        if earlystopper is not None and "early_stopping" in trainer_state:
            earlystopper.load_state_dict(trainer_state["early_stopping"])
        if checkpoint is not None and "checkpoint_min" in trainer_state:
            checkpoint.min_perf_metric = float(trainer_state["checkpoint_min"])
    timer = Timer("train_validate_test")
    timer.start()
    epoch_start = tcfg.get("epoch_start", 0)
    if trainer_state is not None and "epoch_start" not in tcfg and 0 < int(trainer_state.get("epoch", 0)) < num_epoch:
        epoch_start = int(trainer_state["epoch"])  # resume where the saved (unfinished) run stopped
    skipped_seen = 0
    metrics_path = os.path.join("./logs", model_with_config_name, "metrics.jsonl")
    _, rank = get_comm_size_and_rank()
    epoch = epoch_start - 1
    for epoch in range(epoch_start, num_epoch):
        os.environ["HYDRAGNN_EPOCH"] = str(epoch)
        t0 = time.time()
        profiler.set_current_epoch(epoch)
        for ld in (train_loader, val_loader, test_loader):
            if getattr(ld.sampler, "set_epoch", None) is not None:
                ld.sampler.set_epoch(epoch)
        with profiler as prof:
            tr.enable()
            tr.start("train")
            train_loss, train_tasks = train(train_loader, model, optimizer, verbosity, profiler=prof,
                                            compute_grad_energy=compute_grad_energy, step_engine=step_engine)
            tr.stop("train")
            tr.disable()
            if epoch == 0:
                tr.reset()
        _sync_running_stats(model)
        from ..ops import devcheck

        devcheck.check_all()  # device input checks of captured steps (triplet capacity, element ids)
        t_train = time.time() - t0
        sk = getattr(getattr(optimizer, "optim", optimizer), "skipped_steps", None)
        if sk is not None:
            n_skipped = sk()
            if n_skipped > skipped_seen:
                print_distributed(verbosity, f"WARNING: {n_skipped - skipped_seen} training step(s) with a non-finite "
                                             f"loss skipped in epoch {epoch} (NaN/Inf guard)")
                skipped_seen = n_skipped
        if rank == 0:
            from ..utils.metrics import log_json

            ntrain = min(len(train_loader), get_nbatch(train_loader)) * train_loader.batch_size
            log_json(metrics_path, epoch=epoch, train_loss=float(train_loss), train_seconds=t_train,
                     graphs_per_sec_rank0=ntrain / max(t_train, 1e-9))
        if int(os.getenv("HYDRAGNN_VALTEST", "1")) == 0:
            continue
        val_loss, val_tasks = validate(val_loader, model, verbosity, reduce_ranks=True,
                                       compute_grad_energy=compute_grad_energy)
        test_loss, test_tasks, tv, pv = test(test_loader, model, verbosity, reduce_ranks=True,
                                             return_samples=plot_hist_solution,
                                             compute_grad_energy=compute_grad_energy)
        if scheduler is not None:
            scheduler.step(float(val_loss))
        if writer is not None:
            writer.add_scalar("train error", train_loss, epoch)
            writer.add_scalar("validate error", val_loss, epoch)
            writer.add_scalar("test error", test_loss, epoch)
            for k in range(H):
                writer.add_scalar("train error of task" + str(k), train_tasks[k], epoch)
        print_distributed(verbosity, f"Epoch: {epoch:02d}, Train Loss: {float(train_loss):.8f}, "
                                     f"Val Loss: {float(val_loss):.8f}, Test Loss: {float(test_loss):.8f}")
        print_distributed(verbosity, "Tasks Train Loss:", [float(t) for t in train_tasks])
        print_distributed(verbosity, "Tasks Val Loss:", [float(t) for t in val_tasks])
        print_distributed(verbosity, "Tasks Test Loss:", [float(t) for t in test_tasks])
        total_loss["train"][epoch], total_loss["val"][epoch], total_loss["test"][epoch] = \
            train_loss, val_loss, test_loss
        task_loss["train"][epoch], task_loss["val"][epoch], task_loss["test"][epoch] = \
            train_tasks, val_tasks, test_tasks
        if plot_hist_solution and visualizer is not None:
            visualizer.create_scatter_plots(tv, pv, output_names=config["Variables_of_interest"]["output_names"],
                                            iepoch=epoch)
        if checkpoint is not None:
            if checkpoint(model, optimizer, float(reduce_values_ranks(val_loss))):
                print_distributed(verbosity, "Creating Checkpoint: %f" % checkpoint.min_perf_metric)
            print_distributed(verbosity, "Best Performance Metric: %f" % checkpoint.min_perf_metric)
        if earlystopper is not None and earlystopper(float(reduce_values_ranks(val_loss))):
            print_distributed(verbosity,
                              "Early stopping executed at epoch = %d due to val_loss not decreasing" % epoch)
            break
        if trainer_state is not None:
            _record_trainer_state(trainer_state, epoch, scheduler, earlystopper, checkpoint)
            from ..utils.model import save_trainer_state

            save_trainer_state(model_with_config_name, trainer_state)
        if check_time and check_remaining(t0):
            print_distributed(verbosity, "No time left. Early stop.")
            break
    timer.stop()
    if trainer_state is not None:
        trainer_state["epoch"] = epoch + 1
        if earlystopper is not None:
            trainer_state["early_stopping"] = earlystopper.state_dict()
    if create_plots:
        for k in total_loss:
            total_loss[k] = reduce_values_ranks(total_loss[k])
            task_loss[k] = reduce_values_ranks(task_loss[k])
        _, _, tv, pv = test(test_loader, model, verbosity)
        if config["Variables_of_interest"].get("denormalize_output"):
            from ..postprocess.postprocess import output_denormalize

            tv, pv = output_denormalize(config["Variables_of_interest"]["y_minmax"], tv, pv)
        if rank == 0 and visualizer is not None:
            names = config["Variables_of_interest"]["output_names"]
            visualizer.create_plot_global(tv, pv, output_names=names)
            visualizer.create_scatter_plots(tv, pv, output_names=names)
            visualizer.plot_history(total_loss["train"], total_loss["val"], total_loss["test"], task_loss["train"],
                                    task_loss["val"], task_loss["test"], module.loss_weights, names)
