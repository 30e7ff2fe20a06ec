"""Process-group setup and device selection (reference ``hydragnn/utils/distributed/distributed.py``).

One process per GPU.  World size / rank come from torchrun (``RANK``,
``WORLD_SIZE``, ``LOCAL_RANK``), Open MPI (``OMPI_COMM_WORLD_*``) or Slurm
(``SLURM_*``).  Backend: ``HYDRAGNN_BACKEND`` if set, else ``nccl`` (= RCCL
on ROCm, traffic over xGMI inside a node) when a GPU is present, else ``gloo``.
Host-side metadata collectives use a lazily created gloo group so they never
touch the GPU stream.
"""
import os
import re
import subprocess
from datetime import timedelta

import torch
import torch.distributed as dist


def parse_slurm_nodelist(nodelist):
    """'frontier[00001-00002,00005]' -> ['frontier00001', 'frontier00002', 'frontier00005']."""
    out = []
    for m in re.finditer(r"([^,\[]+)(\[([^\]]+)\])?", nodelist):
        prefix, _, rng = m.group(1), m.group(2), m.group(3)
        if rng is None:
            out.append(prefix)
            continue
        for part in rng.split(","):
            if "-" in part:
                a, b = part.split("-")
                w = len(a)
                out += [f"{prefix}{i:0{w}d}" for i in range(int(a), int(b) + 1)]
            else:
                out.append(prefix + part)
    return [x.lstrip(",") for x in out if x.strip(",")]


def init_comm_size_and_rank():
    if os.getenv("WORLD_SIZE") and os.getenv("RANK"):
        return int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    if os.getenv("OMPI_COMM_WORLD_SIZE") and os.getenv("OMPI_COMM_WORLD_RANK"):
        return int(os.environ["OMPI_COMM_WORLD_SIZE"]), int(os.environ["OMPI_COMM_WORLD_RANK"])
    if os.getenv("SLURM_NPROCS") and os.getenv("SLURM_PROCID"):
        return int(os.environ["SLURM_NPROCS"]), int(os.environ["SLURM_PROCID"])
    return 1, 0


def get_comm_size_and_rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def get_local_rank():
    for k in ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID", "PALS_LOCAL_RANKID"):
        if os.getenv(k) is not None:
            return int(os.environ[k])
    return 0


def _default_backend():
    if os.getenv("HYDRAGNN_BACKEND"):
        return os.environ["HYDRAGNN_BACKEND"]
    if dist.is_nccl_available() and torch.cuda.is_available():
        # RCCL needs one GPU per rank; oversubscribed local ranks (e.g. a 3-rank test on a
        # 1-GPU box) fall back to gloo, which also carries CUDA tensors
        local_world = int(os.getenv("LOCAL_WORLD_SIZE", "1"))
        if local_world <= torch.cuda.device_count():
            return "nccl"
    return "gloo"


def rccl_env():
    """RCCL settings for one MI355X node (xGMI, fully connected peers).

    * ``NCCL_GRAPH_REGISTER=0``: the training step captures its gradient all-reduces
      into a hipGraph; with user-buffer registration off, capture is purely local
      (no peer handshake at capture time), so ranks may capture at different times.
    * P2P stays enabled (the reference Frontier scripts' ``NCCL_P2P_DISABLE=1`` is a
      multi-node workaround, SURVEY §5.8, and would route intra-node traffic
      through host memory).
    Existing user settings win."""
    os.environ.setdefault("NCCL_GRAPH_REGISTER", "0")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def setup_ddp(use_deepspeed=False, backend=None):
    """Initialise ``torch.distributed`` (``env://``, 1800 s timeout); returns (world_size, rank)."""
    if dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    world_size, rank = init_comm_size_and_rank()
    backend = backend or _default_backend()
    master_addr = os.getenv("MASTER_ADDR", "127.0.0.1")
    if os.getenv("HYDRAGNN_MASTER_ADDR"):
        master_addr = os.environ["HYDRAGNN_MASTER_ADDR"]
    elif os.getenv("MASTER_ADDR") is None:
        if os.getenv("SLURM_STEP_NODELIST"):
            master_addr = parse_slurm_nodelist(os.environ["SLURM_STEP_NODELIST"])[0]
        elif os.getenv("SLURM_NODELIST"):
            master_addr = parse_slurm_nodelist(os.environ["SLURM_NODELIST"])[0]
    master_port = os.getenv("HYDRAGNN_MASTER_PORT", os.getenv("MASTER_PORT", "8889"))
    os.environ["MASTER_ADDR"] = master_addr
    os.environ["MASTER_PORT"] = str(master_port)
    os.environ["WORLD_SIZE"] = str(world_size)
    os.environ["RANK"] = str(rank)
    os.environ.setdefault("LOCAL_RANK", str(get_local_rank()))
    if backend == "nccl" and torch.cuda.is_available():
        rccl_env()
        torch.cuda.set_device(get_local_rank() % max(torch.cuda.device_count(), 1))
    dist.init_process_group(backend=backend, init_method="env://", timeout=timedelta(seconds=1800),
                            world_size=world_size, rank=rank)
    return world_size, rank


_host_group = None


def host_group():
    """A gloo group for host-side metadata collectives (None when not distributed)."""
    global _host_group
    if not dist.is_initialized():
        return None
    if dist.get_backend() == "gloo":
        return dist.group.WORLD
    if _host_group is None:
        _host_group = dist.new_group(backend="gloo")
    return _host_group


def get_device_name(use_gpu=True, rank_per_model=1, verbosity_level=0, no_prefix=False):
    if not (use_gpu and torch.cuda.is_available()):
        return "cpu"
    n = torch.cuda.device_count()
    local = get_local_rank()
    idx = (local // max(rank_per_model, 1)) % n
    return str(idx) if no_prefix else f"cuda:{idx}"


def get_device(use_gpu=True, rank_per_model=1, verbosity_level=0):
    return torch.device(get_device_name(use_gpu, rank_per_model, verbosity_level))


def get_distributed_model(model, verbosity=0, sync_batch_norm=False, find_unused_parameters=False, **kw):
    """Wrap in our bucketed-overlap DDP (``parallel/ddp.py``) when world_size > 1."""
    from .ddp import DistributedDataParallel, convert_sync_batchnorm

    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return model
    if sync_batch_norm:
        model = convert_sync_batchnorm(model)
    return DistributedDataParallel(model, find_unused_parameters=find_unused_parameters, **kw)


def is_model_distributed(model):
    from .ddp import DistributedDataParallel

    return isinstance(model, (DistributedDataParallel, torch.nn.parallel.DistributedDataParallel))


def print_peak_memory(verbosity_level, prefix):
    from ..utils.print_utils import print_distributed

    if torch.cuda.is_available():
        dev = torch.cuda.current_device()
        print_distributed(verbosity_level, f"{prefix}: {torch.cuda.max_memory_allocated(dev) / 1024 ** 3:.3f} GB")


def nsplit(a, n):
    k, m = divmod(len(a), n)
    return (a[i * k + min(i, m):(i + 1) * k + min(i + 1, m)] for i in range(n))


def comm_reduce(x, op=None, group=None):
    """All-reduce a host/device tensor; host tensors go through the gloo group."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return x
    op = dist.ReduceOp.SUM if op is None else op
    y = x.detach().clone()
    if y.is_cuda:
        dist.all_reduce(y, op=op, group=group)
    else:
        dist.all_reduce(y, op=op, group=group or host_group())
    return y


def timedelta_parse(text):
    """'1-02:03:04' / '02:03:04' / '03:04' -> timedelta."""
    days = 0
    if "-" in text:
        d, text = text.split("-")
        days = int(d)
    parts = [int(p) for p in text.split(":")]
    while len(parts) < 3:
        parts.insert(0, 0)
    h, m, s = parts
    return timedelta(days=days, hours=h, minutes=m, seconds=s)


def check_remaining(t0):
    """Slurm walltime guard: rank 0 queries squeue, broadcasts stop=True when
    the remaining time is shorter than the longest epoch so far (``distributed.py:394-419``)."""
    import time

    should_stop = False
    if os.getenv("SLURM_JOB_ID") and (not dist.is_initialized() or dist.get_rank() == 0):
        try:
            out = subprocess.check_output(["squeue", "-h", "-j", os.environ["SLURM_JOB_ID"], "-o", "%L"],
                                          text=True, timeout=30).strip()
            remaining = timedelta_parse(out).total_seconds()
            should_stop = remaining < (time.time() - t0)
        except Exception:
            should_stop = False
    if dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([int(should_stop)])
        dist.broadcast(t, 0, group=host_group())
        should_stop = bool(t.item())
    return should_stop
