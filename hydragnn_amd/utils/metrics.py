"""Scalar metrics sink (TensorBoard replacement: TensorBoard is not installed).

``ScalarWriter.add_scalar(tag, value, step)`` appends JSON lines to
``<logdir>/scalars.jsonl``; ``log_json`` writes a one-line JSON metrics record
(graphs/s, step time breakdown) per epoch.
"""
import json
import os
import time


class ScalarWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "scalars.jsonl")
        self._f = open(self.path, "a")

    def add_scalar(self, tag, value, step=None):
        rec = {"tag": tag, "value": float(value), "step": step, "time": time.time()}
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def log_json(path, **record):
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(record) + "\n")
