"""Which hipBLASLt kernel (and time) torch picks for each BERT FC GEMM the autotuner may hand to 'mm':
the library kernel names in a steady-state rocprof window do not say which layer they belong to."""
import torch
from torch.profiler import profile, ProfilerActivity

M = 4096
dt = torch.bfloat16


def run(name, fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
    rows = [(e.key, e.device_time_total / max(1, e.count), e.count) for e in prof.key_averages() if e.device_time_total > 0]
    rows.sort(key=lambda r: -r[1] * r[2])
    for k, t, c in rows[:3]:
        print('%-34s %7.1f us x%-3d %s' % (name, t, c // 10 if c >= 10 else c, k[:110]), flush=True)


def main():
    for K, N in [(768, 2304), (768, 3072), (3072, 768), (768, 768)]:
        x = torch.randn(M, K, device='cuda', dtype=dt)
        w = torch.randn(N, K, device='cuda', dtype=dt)
        b = torch.randn(N, device='cuda', dtype=dt)
        dy = torch.randn(M, N, device='cuda', dtype=dt)
        add = torch.randn(M, K, device='cuda', dtype=dt)
        run('fwd %dx%d' % (K, N), lambda: torch.nn.functional.linear(x, w, b))
        run('dgrad %dx%d' % (K, N), lambda: torch.mm(dy, w))
        run('dgrad+add %dx%d' % (K, N), lambda: torch.mm(dy, w).add_(add))
        run('wgrad %dx%d' % (K, N), lambda: torch.mm(dy.t(), x))


if __name__ == '__main__':
    main()
