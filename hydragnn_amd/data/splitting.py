"""Train/validation/test splitting (reference ``preprocess/load_data.py:329-349``,
``utils/datasets/compositional_data_splitting.py:19-156``,
``preprocess/stratified_sampling.py``)."""
import collections
import math
import random

import torch


def split_dataset(dataset, perc_train, stratify_splitting=False):
    if not stratify_splitting:
        perc_val = (1 - perc_train) / 2
        dataset = list(dataset)
        n = len(dataset)
        random.shuffle(dataset)
        a, b = int(n * perc_train), int(n * (perc_train + perc_val))
        return dataset[:a], dataset[a:b], dataset[b:]
    return compositional_stratified_splitting(list(dataset), perc_train)


def create_dataset_categories(dataset):
    max_graph_size = max(d.num_nodes for d in dataset)
    power_ten = math.ceil(math.log10(max(max_graph_size, 2)))
    elements = torch.unique(torch.cat([torch.unique(d.x[:, 0]) for d in dataset]))
    index = {float(e): i for i, e in enumerate(elements.tolist())}
    cats = []
    for d in dataset:
        el, freq = torch.unique(d.x[:, 0], return_counts=True)
        c = 0
        for e, f in zip(el.tolist(), freq.tolist()):
            c += f * (10 ** (power_ten * index[float(e)]))
        cats.append(c)
    return cats


def duplicate_unique_data_samples(dataset, cats):
    counter = collections.Counter(cats)
    singles = {k for k, v in counter.items() if v == 1}
    extra, extra_c = [], []
    for d, c in zip(dataset, cats):
        if c in singles:
            extra.append(d.clone())
            extra_c.append(c)
    return dataset + extra, cats + extra_c


def _partition(train_size, dataset, cats):
    from sklearn.model_selection import StratifiedShuffleSplit

    sss = StratifiedShuffleSplit(n_splits=1, train_size=train_size, random_state=0)
    a_idx, b_idx = next(sss.split(list(range(len(dataset))), cats))
    return [dataset[i] for i in a_idx], [dataset[i] for i in b_idx]


def compositional_stratified_splitting(dataset, perc_train):
    cats = create_dataset_categories(dataset)
    dataset, cats = duplicate_unique_data_samples(dataset, cats)
    train, valtest = _partition(perc_train, dataset, cats)
    vcats = create_dataset_categories(valtest)
    valtest, vcats = duplicate_unique_data_samples(valtest, vcats)
    val, test = _partition(0.5, valtest, vcats)
    return train, val, test


def stratified_subsample(dataset, subsample_percentage):
    """Category = sum_k freq_k * 100^k over sorted element frequencies (``serialized_dataset_loader.py:214-259``)."""
    from sklearn.model_selection import StratifiedShuffleSplit

    cats = []
    for d in dataset:
        fr = torch.bincount(d.x[:, 0].int())
        fr = sorted(fr[fr > 0].tolist())
        cats.append(sum(f * (100 ** i) for i, f in enumerate(fr)))
    sss = StratifiedShuffleSplit(n_splits=1, train_size=subsample_percentage, random_state=0)
    idx, _ = next(sss.split(list(range(len(dataset))), cats))
    return [dataset[i] for i in idx.tolist()]
