"""Task (branch) parallel multi-task model (reference ``hydragnn/models/MultiTaskModelMP.py:12-276``,
SURVEY §2.6 "Task / branch parallel", §3.6).

SC25 multibranch training assigns every rank to ONE dataset/branch.  The shared
encoder (embedding + conv stack) is data-parallel over the whole world; each
branch decoder (``graph_shared[branch-k]`` + the ``branch-k`` entries of every
head) is data-parallel only over the ranks of that branch.  Decoders of other
branches are pruned from the rank's model, so a rank holds and updates only
its own branch.

MI355X mapping: two gradient communicators — the world group and the branch
group — each driving our bucketed, backward-overlapped all-reduce
(``parallel/ddp.py``) over its own parameter subset (RCCL over xGMI inside a
node).  No encoder/decoder module copies are made: the wrappers hold
references into the base model, so ``state_dict`` keeps the reference layout.
"""
import contextlib

import torch
import torch.distributed as dist
from torch import nn

from ..parallel.ddp import DistributedDataParallel
from ..utils import tracer as tr

_DECODER_ROOTS = ("graph_shared", "heads_NN", "convs_node_hidden", "convs_node_output", "batch_norms_node_hidden",
                  "batch_norms_node_output")


class _Params(nn.Module):
    """A parameter-only view: registers references to a subset of a model's submodules."""

    def __init__(self, named_modules):
        super().__init__()
        for name, m in named_modules:
            self.add_module(name.replace(".", "__"), m)

    def forward(self, *a, **k):  # never called: the base model runs the forward
        raise RuntimeError("parameter view")


def split_encoder_decoder(model):
    enc, dec = [], []
    for name, child in model.named_children():
        (dec if name in _DECODER_ROOTS else enc).append((name, child))
    return enc, dec


def prune_branches(model, branch_id):
    """Delete every decoder branch except ``branch-{branch_id}`` (reference ``MultiTaskModelMP.py:203-217``)."""
    keep = f"branch-{branch_id}"
    for k in [k for k in model.graph_shared.keys() if k != keep]:
        del model.graph_shared[k]
    for head in model.heads_NN:
        for k in [k for k in head.keys() if k != keep]:
            del head[k]
    for dname in ("convs_node_hidden", "convs_node_output", "batch_norms_node_hidden", "batch_norms_node_output"):
        d = getattr(model, dname, None)
        if d is not None:
            for k in [k for k in d.keys() if k != keep]:
                del d[k]


class MultiTaskModelMP(nn.Module):
    """``MultiTaskModelMP(base_model, group_color, head_pg)`` — same constructor as the reference."""

    def __init__(self, base_model, group_color, head_pg, bucket_cap_mb=25.0):
        super().__init__()
        self.shared_pg = dist.group.WORLD
        self.head_pg = head_pg
        self.shared_pg_size = dist.get_world_size(self.shared_pg)
        self.shared_pg_rank = dist.get_rank(self.shared_pg)
        self.head_pg_size = dist.get_world_size(head_pg)
        self.head_pg_rank = dist.get_rank(head_pg)
        self.branch_id = int(group_color)
        prune_branches(base_model, self.branch_id)
        self.module = base_model
        enc, dec = split_encoder_decoder(base_model)
        self.encoder = DistributedDataParallel(_Params(enc), process_group=self.shared_pg,
                                               bucket_cap_mb=bucket_cap_mb, find_unused_parameters=True)
        self.decoder = DistributedDataParallel(_Params(dec), process_group=self.head_pg,
                                               bucket_cap_mb=bucket_cap_mb, find_unused_parameters=True)

    def forward(self, data):
        tr.start("enc_forward")
        x, equiv, ctx = self.module.encode(data)
        tr.stop("enc_forward")
        tr.start(f"branch{self.branch_id}_forward")
        out = self.module.decode(x, equiv, ctx)
        tr.stop(f"branch{self.branch_id}_forward")
        return out

    def parameters(self, recurse=True):
        return self.module.parameters(recurse)

    def named_parameters(self, prefix="", recurse=True, remove_duplicate=True):
        return self.module.named_parameters(prefix, recurse, remove_duplicate)

    def state_dict(self, *a, **k):
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, sd, strict=True):
        return self.module.load_state_dict(sd, strict=strict)

    def zero_grad(self, set_to_none=False):
        self.encoder.zero_grad()
        self.decoder.zero_grad()

    @contextlib.contextmanager
    def no_sync(self):
        """Skip both gradient synchronisations (reference ``--nosync``, ``MultiTaskModelMP.py:262-276``)."""
        with self.encoder.no_sync(), self.decoder.no_sync():
            yield

    def loss(self, *a, **k):
        return self.module.loss(*a, **k)

    def energy_force_loss(self, *a, **k):
        return self.module.energy_force_loss(*a, **k)


def branch_groups_mesh(num_branches, device_type=None):
    """Device-mesh variant of :func:`branch_groups` (reference ``examples/multibranch/
    train.py:216-252``, ``--use_devicemesh``): a 2-D ``init_device_mesh`` of shape
    (branches, world // branches); the first mesh coordinate is the branch id, the
    second dimension's group (ranks of one branch) is the branch group.  Equal split,
    so ``world`` must be a multiple of the branch count.

    Returns (branch_id_of_this_rank, this_branch_group, rank_lists)."""
    from torch.distributed.device_mesh import init_device_mesh

    world = dist.get_world_size()
    assert world % num_branches == 0, f"device mesh: world {world} is not a multiple of {num_branches} branches"
    if device_type is None:
        device_type = "cuda" if dist.get_backend() == "nccl" else "cpu"
    mesh = init_device_mesh(device_type, (num_branches, world // num_branches), mesh_dim_names=("branch", "replica"))
    bid = mesh.get_coordinate()[0]
    per = world // num_branches
    lists = [list(range(b * per, (b + 1) * per)) for b in range(num_branches)]
    return bid, mesh["replica"].get_group(), lists


def branch_groups(sizes, world=None, rank=None):
    """Assign ranks to branches proportionally to ``sizes`` (e.g. dataset sizes; every branch
    gets >= 1 rank) and create one process group per branch (reference
    ``examples/multibranch/train.py:183-189, 253-279``).

    Returns (branch_id_of_this_rank, this_branch_group, rank_lists)."""
    world = dist.get_world_size() if world is None else world
    rank = dist.get_rank() if rank is None else rank
    nb = len(sizes)
    assert world >= nb, f"need at least one rank per branch ({nb} branches, world {world})"
    tot = float(sum(sizes))
    counts = [1] * nb
    for _ in range(world - nb):  # largest remaining deficit gets the next rank (deterministic)
        deficit = [sizes[i] / tot * world - counts[i] for i in range(nb)]
        counts[max(range(nb), key=lambda i: deficit[i])] += 1
    lists, r0 = [], 0
    for c in counts:
        lists.append(list(range(r0, r0 + c)))
        r0 += c
    groups = [dist.new_group(ranks=l) for l in lists]  # every rank must create every group
    bid = next(i for i, l in enumerate(lists) if rank in l)
    return bid, groups[bid], lists
