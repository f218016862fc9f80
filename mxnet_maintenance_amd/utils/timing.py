"""Wall-clock and device-event timing helpers used by benchmarks and the autotuner."""
import time

import torch


class Timer:
    """``with Timer(sync=True) as t: ...; t.ms``: synchronises the device on both sides when on GPU."""

    def __init__(self, sync=True):
        self.sync = sync and torch.cuda.is_available()
        self.ms = 0.0

    def __enter__(self):
        if self.sync:
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self.sync:
            torch.cuda.synchronize()
        self.ms = (time.perf_counter() - self._t0) * 1000.0
        return False


def cuda_time(fn, iters=10, warmup=2):
    """Mean milliseconds of ``fn()`` measured with HIP events on the current stream."""
    for _ in range(warmup):
        fn()
    if not torch.cuda.is_available():
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        return (time.perf_counter() - t0) * 1000.0 / iters
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters
