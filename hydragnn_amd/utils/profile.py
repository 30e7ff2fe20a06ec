"""torch.profiler wrapper (reference ``utils/profiling_and_tracing/profile.py:9-70``).

``"Profile": {"enable": 1, "target_epoch": k}`` profiles epoch k with the
schedule wait=5, warmup=3, active=3 and writes a Chrome trace to the log dir
(TensorBoard is not installed).  On ROCm the CUDA activity is HIP activity
(roctracer).  Disabled -> a null context whose ``step()`` is a no-op.
"""
import os

import torch


class _Null:
    def step(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class Profiler:
    def __init__(self, prefix="./logs/profile", enable=False, target_epoch=0):
        self.prefix = prefix
        self.enable = enable
        self.target_epoch = target_epoch
        self.current_epoch = -1
        self._prof = None

    def setup(self, config):
        self.enable = bool(config.get("enable", 0))
        self.target_epoch = int(config.get("target_epoch", 0))

    def set_current_epoch(self, e):
        self.current_epoch = e

    def _handler(self, prof):
        os.makedirs(self.prefix, exist_ok=True)
        prof.export_chrome_trace(os.path.join(self.prefix, f"trace_epoch{self.current_epoch}.json"))

    def __enter__(self):
        if not (self.enable and self.current_epoch == self.target_epoch):
            self._prof = None
            return _Null()
        acts = [torch.profiler.ProfilerActivity.CPU]
        if torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self._prof = torch.profiler.profile(activities=acts,
                                            schedule=torch.profiler.schedule(wait=5, warmup=3, active=3),
                                            on_trace_ready=self._handler, record_shapes=True, with_stack=True)
        self._prof.__enter__()
        return self._prof

    def __exit__(self, *a):
        if self._prof is not None:
            self._prof.__exit__(*a)
            self._prof = None
        return False
