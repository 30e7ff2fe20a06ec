"""Rank-aware logging with the reference verbosity levels (``utils/print/print_utils.py``).

Verbosity: 0 nothing; 1 rank 0 basic; 2 rank 0 + progress bars; 3 all ranks
basic; 4 all ranks + progress bars.  Log file: ``./logs/<name>/run.log``
with a ``"<rank>: "`` prefix.
"""
import logging
import os

import torch.distributed as dist

try:
    from tqdm import tqdm
except ImportError:  # pragma: no cover
    tqdm = None


def _rank():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank()
    for k in ("RANK", "OMPI_COMM_WORLD_RANK", "SLURM_PROCID"):
        if k in os.environ:
            return int(os.environ[k])
    return 0


def print_nothing(*args):
    pass


def print_master(*args):
    log(*args, rank=0)


def print_all_processes(*args):
    log(*args)


switcher = {0: print_nothing, 1: print_master, 2: print_master, 3: print_all_processes, 4: print_all_processes}


def print_distributed(verbosity_level, *args):
    return switcher.get(verbosity_level, print_nothing)(*args)


def iterate_tqdm(iterator, verbosity_level, *args, **kwargs):
    if tqdm is not None and ((_rank() == 0 and verbosity_level == 2) or verbosity_level == 4):
        return tqdm(iterator, *args, **kwargs)
    return iterator


def setup_log(prefix, path="./logs"):
    rank = _rank()
    fmt = logging.Formatter("%d: %%(message)s" % rank)
    logger = logging.getLogger("hydragnn")
    logger.propagate = False
    logger.setLevel(logging.DEBUG)
    os.makedirs(os.path.join(path, prefix), exist_ok=True)
    if logger.hasHandlers():
        logger.handlers.clear()
    fh = logging.FileHandler(os.path.join(path, prefix, "run.log"))
    fh.setFormatter(fmt)
    logger.addHandler(fh)
    ch = logging.StreamHandler()
    ch.setFormatter(fmt)
    logger.addHandler(ch)


def log(*args, sep=" ", rank=None):
    logger = logging.getLogger("hydragnn")
    if rank is None or rank == _rank():
        logger.info(sep.join(map(str, args)))


def log0(*args, sep=" "):
    log(*args, sep=sep, rank=0)
