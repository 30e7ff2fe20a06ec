"""ZeRO-1 optimizer-state sharding (reference: ``torch.distributed.optim.ZeroRedundancyOptimizer``
selected by ``Optimizer.use_zero_redundancy``, ``utils/optimizer/optimizer.py:43-113``).

Parameters are partitioned greedily by size over the ranks; every rank keeps
optimizer state only for its shard and steps it, then each owner broadcasts its
updated shard as ONE packed buffer (world_size collectives per step, not one
per tensor).  ``consolidate_state_dict()`` gathers the full state to rank 0 for
checkpointing (reference ``model.py:67-68``).
"""
import torch
import torch.distributed as dist


class ZeroRedundancyOptimizer(torch.optim.Optimizer):
    def __init__(self, params, optimizer_factory, process_group=None):
        params = list(params)
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        sizes = [0] * self.world
        self.owner = {}
        self.shards = [[] for _ in range(self.world)]
        for p in sorted(params, key=lambda t: -t.numel()):
            r = min(range(self.world), key=lambda k: sizes[k])
            sizes[r] += p.numel()
            self.shards[r].append(p)
            self.owner[p] = r
        self.all_params = params
        local = self.shards[self.rank]
        self.optim = optimizer_factory(local) if local else None
        super().__init__(params, {"lr": self.optim.defaults["lr"] if self.optim else 0.0})
        if self.optim is not None:
            # share hyper-parameters so schedulers acting on this wrapper reach the inner optimizer
            self.param_groups[0]["lr"] = self.optim.param_groups[0]["lr"]
        self._consolidated = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self.optim is not None:
            for g in self.optim.param_groups:
                g["lr"] = self.param_groups[0]["lr"]
            self.optim.step()
        if self.world > 1:
            for r in range(self.world):
                ps = self.shards[r]
                if not ps:
                    continue
                flat = torch.cat([p.data.reshape(-1) for p in ps])
                dist.broadcast(flat, src=r if self.group is None else dist.get_global_rank(self.group, r),
                               group=self.group)
                off = 0
                for p in ps:
                    p.data.copy_(flat[off:off + p.numel()].view_as(p))
                    off += p.numel()
        return loss

    def zero_grad(self, set_to_none=True):
        for p in self.all_params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def consolidate_state_dict(self, to=0):
        """Gather every shard's optimizer state on rank ``to``."""
        local = self.optim.state_dict() if self.optim is not None else None
        if self.world == 1:
            self._consolidated = [local]
            return
        objs = [None] * self.world
        dist.all_gather_object(objs, local, group=self.group)
        self._consolidated = objs if self.rank == to else None

    def state_dict(self):
        if self._consolidated is not None:
            return {"shards": self._consolidated, "param_groups": self.param_groups_meta()}
        return {"shards": [self.optim.state_dict() if self.optim is not None else None],
                "param_groups": self.param_groups_meta()}

    def param_groups_meta(self):
        return [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]

    def load_state_dict(self, state):
        shards = state.get("shards", [])
        if self.optim is not None:
            mine = shards[self.rank] if len(shards) == self.world else (shards[0] if shards else None)
            if mine is not None:
                self.optim.load_state_dict(mine)
