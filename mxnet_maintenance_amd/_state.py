"""Thread-local imperative state: autograd recording / training flags.

Parity: src/imperative/imperative.cc (Imperative::is_recording_, is_training_,
is_np_shape_). Kept in its own module so ops can read the flags without
importing the autograd front-end.
"""
import threading


class _State(threading.local):
    def __init__(self):
        super().__init__()
        self.recording = False
        self.training = False
        self.np_shape = False
        self.np_array = False
        # NDArrays marked with attach_grad that were consumed while recording,
        # keyed by id -> NDArray.  Cleared by backward() (unless retain_graph).
        self.tape_leaves = {}


STATE = _State()

# >0 while mx.autograd.backward runs (plain, no create_graph): backward kernels may
# accumulate parameter gradients straight into the leaves' .grad buffers.  Process-wide
# (not thread-local) because torch runs GPU backward functions on its device threads.
DIRECT_GRAD = [0]


def is_recording():
    return STATE.recording


def is_training():
    return STATE.training

# HIP-graph capture of a training step (gluon.GraphStep): a device uint64 counter mixed into the seeds of
# captured dropout kernels, advanced before every replay so masks differ between replays
GRAPH_RNG = [None]


# ids of NDArray leaves whose gradient buffer a backward pass actually reached (filled by the
# post-accumulate hook NDArray.attach_grad registers; read when marking gradients fresh)
GRAD_TOUCHED = set()
