"""Does the autotuner's short timing (3 calls x 2 rounds) measure kernels or host launch overhead?
Times hipBLASLt and the in-tree candidates of the BERT FFN GEMM both ways and reports the host cost
per call of each Python launch path."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402
from mxnet_maintenance_amd.ops import gemm as G  # noqa: E402


def ev_time(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def ev_time_sleep(fn, reps, cycles=2_000_000):
    """The GPU is held by a sleep kernel while the calls are enqueued: back-to-back kernel time only."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(cycles)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def host_time(fn, reps=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / reps * 1e6


M, K, N = 4096, 768, 3072
x = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
w = torch.randn(N, K, device='cuda', dtype=torch.bfloat16) * 0.05
cands = {
    'mm': lambda: torch.nn.functional.linear(x, w),
    'hip26': lambda: KF.conv_fwd(x.view(M, 1, 1, K), w.view(N, 1, 1, K), (1, 1), (0, 0), None, 26).view(M, N),
    'gemm1s1': lambda: G.gemm_nt(x, w, cfg=(1, 1)),
}
for n, f in cands.items():
    f()
torch.cuda.synchronize()
s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s0.record()
torch.cuda._sleep(2_000_000)
e0.record()
e0.synchronize()
print('_sleep(2e6 cycles) = %.1f us' % (s0.elapsed_time(e0) * 1e3))
for n, f in cands.items():
    short = min(ev_time(f, 3) for _ in range(2))
    slept = min(ev_time_sleep(f, 3) for _ in range(2))
    long_ = ev_time(f, 50)
    print('%-8s autotune-style %.1f us   behind a sleep %.1f us   50 reps %.1f us   host %.1f us/call'
          % (n, short, slept, long_, host_time(f)), flush=True)
