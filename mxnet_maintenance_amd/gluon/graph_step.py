"""HIP-graph capture of a whole training (or inference) step.

The reference amortises per-operator launch cost with a static computation
graph executed by its C++ engine (``hybridize(static_alloc=True,
static_shape=True)``, CachedOp: src/imperative/cached_op.cc) and, on NVIDIA,
with CUDA graphs inside that executor (src/imperative/cuda_graphs.h).  On
MI355X the same effect comes from capturing the *entire* step -- forward,
backward, gradient reduction and the fused optimizer update -- into one HIP
graph and replaying it: one host call launches thousands of kernels, so a
launch-bound model (BERT at small per-GPU batch) runs at kernel speed.

What changes between replays lives on the device:

* optimizer hyper-parameters (learning rate from the scheduler, Adam/LAMB
  bias corrections) -- the trainer writes them into a small device table
  before every replay (``Trainer._stage_hyper``) and the fused kernels read
  them through a pointer captured in the graph;
* dropout masks -- captured dropout kernels add a device counter, bumped
  before each replay, to their Philox key;
* torch's own generator (``nd.random`` ops) is graph-safe by construction.

Data parallel (one process per GPU): the trainer's gradient-bucket hooks fire
during the captured backward and issue their RCCL all-reduces from the
capturing stream; ProcessGroupNCCL runs them on its own stream, which joins
the capture through events, so every replay launches forward, the overlapped
bucket all-reduces, the tail reduces and the update as one graph.  All ranks
capture at the same call (warm-up counts are identical), and the eager
warm-up steps have already created the communicators.

Usage::

    def train_step(data, label):
        with autograd.record():
            loss = loss_fn(net(data), label)
        loss.backward()
        trainer.step(batch_size)
        return loss

    step = gluon.GraphStep(train_step, trainer, warmup=3)
    for data, label in loader:
        loss = step(data, label)      # same shapes every call

The first ``warmup`` calls run eagerly (kernel autotuning, lazy parameter
initialisation and gradient-arena construction happen there), the next call
captures and replays.  Inputs are copied into static buffers; returned
arrays are the graph's static outputs and are overwritten by the next call.
The step function must not read device values on the host (``asnumpy``,
``asscalar``) and must be shape-stable; AMP dynamic loss scaling (a host-side
overflow check) is not supported inside a captured step.
"""
import gc
import os

import torch

from .. import _state
from ..ndarray.ndarray import NDArray

__all__ = ['GraphStep']


def _tensor_of(x):
    return x._data if isinstance(x, NDArray) else x


class GraphStep:
    """Capture ``fn(*inputs)`` into a HIP graph after ``warmup`` eager calls, then replay it."""

    def __init__(self, fn, trainer=None, warmup=3, fallback=False):
        if warmup < 1:
            raise ValueError('GraphStep needs at least one eager warm-up call')
        self._fn = fn
        self._trainer = trainer
        self._warmup = int(warmup)
        self._calls = 0
        self._graph = None
        self._static_in = None
        self._static_out = None
        self._stream = None
        self._rng = None
        self._fallback = fallback     # capture failure -> keep running eagerly (with a warning)
        self._eager_only = False

    @property
    def captured(self):
        return self._graph is not None

    def _side_stream(self, device):
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=device)
        return self._stream

    @staticmethod
    def _device(inputs):
        dev = next((_tensor_of(x).device for x in inputs if torch.is_tensor(_tensor_of(x))), None)
        if dev is None and torch.cuda.is_available():      # closure-only step: the current device
            dev = torch.device('cuda', torch.cuda.current_device())
        return dev

    def _run_eager(self, inputs):
        dev = self._device(inputs)
        if dev is None or dev.type != 'cuda':
            return self._fn(*inputs)
        s = self._side_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            out = self._fn(*inputs)
        torch.cuda.current_stream(dev).wait_stream(s)
        return out

    def _capture(self, inputs):
        tin = [_tensor_of(x) for x in inputs]
        dev = self._device(inputs)
        if dev is None or dev.type != 'cuda':
            raise RuntimeError('GraphStep captures HIP work: inputs must live on a GPU context')
        # tensors get static device buffers; other arguments (ints, flags) are captured as constants
        self._static_in = [NDArray(t.clone()) if isinstance(x, NDArray) else (t.clone() if torch.is_tensor(t) else x)
                           for x, t in zip(inputs, tin)]
        self._rng = torch.zeros(1, dtype=torch.int64, device=dev)
        if self._trainer is not None:
            self._trainer._enter_graph_mode()
        s = self._side_stream(dev)
        if os.environ.get('MXAMD_GRAPH_GC', '1') == '1':
            gc.collect()
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        _state.GRAPH_RNG[0] = self._rng
        try:
            with torch.cuda.graph(graph, stream=s):
                self._static_out = self._fn(*self._static_in)
        except Exception:
            if self._trainer is not None:
                self._trainer._exit_graph_mode()
            raise
        finally:
            _state.GRAPH_RNG[0] = None
        self._graph = graph

    def _load_inputs(self, inputs):
        if len(inputs) != len(self._static_in):
            raise ValueError('GraphStep: expected %d inputs, got %d' % (len(self._static_in), len(inputs)))
        for dst, src in zip(self._static_in, inputs):
            d, t = _tensor_of(dst), _tensor_of(src)
            if not torch.is_tensor(d):
                if d != t:
                    raise ValueError('GraphStep: non-tensor argument %r differs from the captured %r' % (t, d))
                continue
            if d.shape != t.shape or d.dtype != t.dtype:
                raise ValueError('GraphStep: input %s/%s differs from the captured %s/%s'
                                 % (tuple(t.shape), t.dtype, tuple(d.shape), d.dtype))
            if d.data_ptr() != t.data_ptr():
                d.copy_(t, non_blocking=True)

    @property
    def static_inputs(self):
        """The captured input buffers: fill them in place to skip the copy in ``__call__``."""
        return self._static_in

    def __call__(self, *inputs):
        self._calls += 1
        if self._eager_only:
            return self._run_eager(inputs)
        if self._graph is None:
            if self._calls <= self._warmup:
                return self._run_eager(inputs)
            err = None
            try:
                self._capture(inputs)
            except Exception as e:      # pylint: disable=broad-except
                err = e
            # data parallel: the ranks decide TOGETHER -- one rank replaying a graph while another
            # runs eagerly would pair their collectives differently (hang risk)
            if not self._all_ranks_ok(err is None):
                if self._graph is not None:
                    self._drop_graph()
                if not self._fallback:
                    raise err if err is not None else RuntimeError('GraphStep: capture failed on another rank')
                import warnings
                warnings.warn('GraphStep: capture failed (%s); running the step eagerly on every rank'
                              % (err if err is not None else 'on another rank'))
                self._eager_only = True
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                return self._run_eager(inputs)
        else:
            self._load_inputs(inputs)
        if self._trainer is not None:
            self._trainer._stage_hyper()
        self._rng.add_(1)
        self._graph.replay()
        return self._static_out

    @staticmethod
    def _all_ranks_ok(ok):
        """MIN over ranks of a success flag (CPU collective; True with one process)."""
        from ..parallel import dist
        if dist.world_size() <= 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op='min')
        return bool(t.item())

    def _drop_graph(self):
        if self._trainer is not None:
            self._trainer._exit_graph_mode()
        self._graph = None
        self._static_out = None

    def reset(self):
        """Drop the captured graph (e.g. after a shape change); the next call re-captures."""
        if self._trainer is not None and self._graph is not None:
            self._trainer._exit_graph_mode()
        self._graph = None
        self._static_out = None
        self._static_in = None
        self._calls = self._warmup
