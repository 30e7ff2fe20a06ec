"""Hyper-parameter-optimisation launch helpers (reference ``hydragnn/utils/hpo/deephyper.py:5-177``,
SURVEY P43; drivers in ``examples/qm9_hpo``, ``examples/multidataset_hpo``).

The reference launches each trial as an ``srun`` sub-job on a Slurm allocation of
Frontier nodes (plus a DeepSpeed config writer and an unrelated Megatron template).
On one MI355X node the natural unit is a *GPU slot*: the 8 GPUs are partitioned into
``8 / gpus_per_trial`` slots and every trial runs as a ``torchrun`` child process
restricted to its slot via ``HIP_VISIBLE_DEVICES``, with its own rendezvous port.

* :func:`read_node_list`, :func:`master_from_host` — allocation introspection (Slurm);
* :func:`create_launch_command` — the ``torchrun`` command line of one trial;
* :class:`TrialScheduler` — runs trials concurrently on disjoint GPU slots and
  collects each trial's last JSON line (the examples print their result dict);
* :func:`random_search` — a minimal search loop over a parameter space
  (DeepHyper/Optuna are not installed; any external optimiser can drive
  :class:`TrialScheduler` instead).
"""
import itertools
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

from ..parallel.distributed import parse_slurm_nodelist


def read_node_list():
    """Nodes of the allocation.  The reference decodes ``SLURM_NODELIST`` per machine
    (``HYDRAGNN_SYSTEM`` = frontier / perlmutter fixed-width prefixes); the bracket-range
    parser here is prefix- and width-generic, so ``HYDRAGNN_SYSTEM`` needs no value."""
    nl = os.environ.get("SLURM_NODELIST", socket.gethostname())
    nodes = parse_slurm_nodelist(nl)
    return nodes, ",".join(nodes)


def master_from_host(host):
    return socket.gethostbyname(host)


def create_launch_command(script, args=(), nproc=1, master_port=29500, python=None, master_addr="127.0.0.1"):
    py = python or sys.executable
    return [py, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}", "--master-addr",
            master_addr, f"--master-port={master_port}", script] + [str(a) for a in args]


def _last_json(text):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except json.JSONDecodeError:
                continue
    return None


class TrialScheduler:
    """Run trials on disjoint GPU slots of one node.  ``submit(args)`` queues a trial
    (script arguments); ``run()`` executes everything, at most one trial per slot at a time."""

    def __init__(self, script, total_gpus=8, gpus_per_trial=1, base_port=29600, workdir=".", env=None,
                 timeout=None):
        assert total_gpus % gpus_per_trial == 0, "gpus_per_trial must divide total_gpus"
        self.script, self.g = script, gpus_per_trial
        self.slots = [list(range(s, s + gpus_per_trial)) for s in range(0, total_gpus, gpus_per_trial)]
        self.base_port, self.workdir, self.env, self.timeout = base_port, workdir, env or {}, timeout
        self.queue, self.results = [], []

    def submit(self, args):
        self.queue.append(list(args))
        return len(self.queue) - 1

    def run(self, poll=0.5):
        pending = list(enumerate(self.queue))
        running = {}  # slot -> (trial id, Popen, start, log path)
        results = [None] * len(self.queue)
        port = itertools.count(self.base_port)
        while pending or running:
            for s in range(len(self.slots)):
                if s not in running and pending:
                    tid, args = pending.pop(0)
                    d = os.path.join(self.workdir, f"trial_{tid}")
                    os.makedirs(d, exist_ok=True)
                    env = dict(os.environ, **self.env,
                               HIP_VISIBLE_DEVICES=",".join(str(g) for g in self.slots[s]))
                    # each trial's torchrun owns its rendezvous port: an inherited port override
                    # would put concurrent trials on one port
                    env.pop("HYDRAGNN_MASTER_PORT", None)
                    cmd = create_launch_command(self.script, list(args) + ["--workdir", d], self.g, next(port))
                    log = open(os.path.join(d, "trial.log"), "w")
                    p = subprocess.Popen(cmd, cwd=d, env=env, stdout=log, stderr=subprocess.STDOUT, text=True)
                    running[s] = (tid, p, time.time(), log)
            for s, (tid, p, t0, log) in list(running.items()):
                expired = self.timeout is not None and time.time() - t0 > self.timeout
                if p.poll() is None and not expired:
                    continue
                if expired and p.poll() is None:
                    p.kill()
                    p.wait()
                log.close()
                with open(log.name) as f:
                    out = f.read()
                results[tid] = {"returncode": p.returncode, "result": _last_json(out), "log": log.name}
                del running[s]
            time.sleep(poll)
        self.results = results
        return results


def random_search(space, n_trials, scheduler, objective="test_error", seed=0, fixed_args=()):
    """Sample ``n_trials`` points of ``space`` ({"--flag": [choices]}), run them through
    ``scheduler`` and return (best_args, best_value, all results)."""
    rng = np.random.default_rng(seed)
    trials = []
    for _ in range(n_trials):
        args = list(fixed_args)
        for flag, choices in space.items():
            args += [flag, choices[int(rng.integers(len(choices)))]]
        trials.append(args)
        scheduler.submit(args)
    res = scheduler.run()
    scored = [(r["result"][objective], a) for r, a in zip(res, trials)
              if r["returncode"] == 0 and r["result"] and objective in r["result"]]
    if not scored:
        return None, None, res
    best = min(scored, key=lambda t: t[0])
    return best[1], best[0], res
