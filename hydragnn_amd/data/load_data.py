"""Dataset loading, splitting and loader construction (reference ``preprocess/load_data.py:206-438``).

``dataset_loading_and_splitting(config)``:
  raw directories -> (rank 0) ``RawDataLoader`` -> normalised serialized files -> barrier;
  a "total" split -> ``split_dataset`` (random | compositional-stratified) -> 3 files;
  then ``SerializedDataLoader`` for train/validate/test and ``create_dataloaders``.
"""
import os

import torch.distributed as dist

from ..parallel.distributed import get_comm_size_and_rank
from ..utils.time_utils import Timer
from .loader import DeviceGraphLoader, GraphDataLoader, make_sampler
from .lsms import RawDataLoader
from .serialized import SerializedDataLoader, read_serialized, write_serialized
from .splitting import split_dataset


def _serialized_dir():
    return os.path.join(os.environ.get("SERIALIZED_DATA_PATH", os.getcwd()), "serialized_dataset")


def dataset_loading_and_splitting(config):
    if not list(config["Dataset"]["path"].values())[0].endswith(".pkl"):
        transform_raw_data_to_serialized(config["Dataset"])
    if "total" in config["Dataset"]["path"].keys():
        total_to_train_val_test_pkls(config)
    trainset, valset, testset = load_train_val_test_sets(config)
    return create_dataloaders(trainset, valset, testset, batch_size=config["NeuralNetwork"]["Training"]["batch_size"])


def create_dataloaders(trainset, valset, testset, batch_size, train_sampler_shuffle=True, val_sampler_shuffle=True,
                       test_sampler_shuffle=True, group=None, oversampling=False, num_samples=None, local=False):
    """``local=True``: every rank already holds its own shard (multidataset subsets), so
    the samplers shuffle the local data without sharding it again across ranks."""
    ns = num_samples or (None, None, None)
    if local:
        from .loader import _ShuffleSampler

        return tuple(GraphDataLoader(ds, batch_size, sampler=_ShuffleSampler(len(ds), sh))
                     for ds, sh in ((trainset, train_sampler_shuffle), (valset, val_sampler_shuffle),
                                    (testset, test_sampler_shuffle)))
    tr = GraphDataLoader(trainset, batch_size, sampler=make_sampler(trainset, train_sampler_shuffle, group,
                                                                    oversampling, ns[0]))
    va = GraphDataLoader(valset, batch_size, sampler=make_sampler(valset, val_sampler_shuffle, group, oversampling,
                                                                  ns[1]))
    te = GraphDataLoader(testset, batch_size, sampler=make_sampler(testset, test_sampler_shuffle, group,
                                                                   oversampling, ns[2]))
    return tr, va, te


def to_device_loaders(loaders, device, head_types, head_dims, attn_scope="batch"):
    """Move every split into HBM (``DeviceGraphStore``) keeping the samplers."""
    from .device_store import DeviceGraphStore

    out = []
    for ld in loaders:
        store = DeviceGraphStore(list(ld.dataset), device, head_types=head_types, head_dims=head_dims,
                                 attn_scope=attn_scope)
        out.append(DeviceGraphLoader(ld.dataset, store, ld.batch_size, sampler=ld.sampler))
    return out


def load_train_val_test_sets(config, isdist=False):
    timer = Timer("load_data")
    timer.start()
    sets = {}
    for split, path in config["Dataset"]["path"].items():
        f = path if path.endswith(".pkl") else os.path.join(_serialized_dir(), f"{config['Dataset']['name']}_{split}.pkl")
        sets[split] = SerializedDataLoader(config, dist=isdist).load_serialized_data(f)
    timer.stop()
    return sets["train"], sets["validate"], sets["test"]


def transform_raw_data_to_serialized(dataset_config):
    _, rank = get_comm_size_and_rank()
    if rank == 0:
        if dataset_config["format"] not in ("LSMS", "unit_test", "CFG", "XYZ"):
            raise NameError("Data format not recognized for raw data loader")
        RawDataLoader(dataset_config).load_raw_data(_serialized_dir())
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def total_to_train_val_test_pkls(config, isdist=False):
    _, rank = get_comm_size_and_rank()
    p = config["Dataset"]["path"]
    f = p["total"] if list(p.values())[0].endswith(".pkl") else os.path.join(_serialized_dir(),
                                                                            config["Dataset"]["name"] + ".pkl")
    mn, mg, total = read_serialized(f)
    tr, va, te = split_dataset(total, config["NeuralNetwork"]["Training"]["perc_train"],
                               config["Dataset"].get("compositional_stratified_splitting", False))
    d = os.path.dirname(f)
    config["Dataset"]["path"] = {}
    for split, ds in zip(("train", "validate", "test"), (tr, va, te)):
        name = os.path.join(d, config["Dataset"]["name"] + "_" + split + ".pkl")
        config["Dataset"]["path"][split] = name
        if isdist or rank == 0:
            write_serialized(name, ds, mn, mg)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
