"""GEMM microbench on the BERT-base / ResNet FC shapes: hipBLASLt (torch) against every in-tree MFMA
candidate (conv kernels on a 1x1 image, the dedicated GEMM kernel when built), TF/s per candidate.

    python tools/bench_gemm.py [--tokens 4096] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402
from mxnet_maintenance_amd.ops import kernels as _K  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tokens', type=int, default=4096)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    M = a.tokens
    dt = torch.bfloat16
    shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]     # (K in, N out) of BERT-base
    tot = {}
    for K, N in shapes:
        x = torch.randn(M, K, device='cuda', dtype=dt)
        w = torch.randn(N, K, device='cuda', dtype=dt) * 0.05
        dy = torch.randn(M, N, device='cuda', dtype=dt)
        fl = 2.0 * M * N * K
        ref_f = torch.nn.functional.linear(x.float(), w.float())
        ref_d = dy.float() @ w.float()
        cands = {'fwd': [('mm', lambda: torch.nn.functional.linear(x, w))],
                 'dgrad': [('mm', lambda: torch.mm(dy, w))],
                 'wgrad': [('mm', lambda: torch.mm(dy.t(), x))]}
        for v in KF._fwd_variants(K, N):
            cands['fwd'].append(('conv%d' % v, lambda v=v: KF.conv_fwd(x.view(M, 1, 1, K), w.view(N, 1, 1, K),
                                                                       (1, 1), (0, 0), None, v).view(M, N)))
        wt = w.t().contiguous()
        for v in KF._fwd_variants(N, K):
            cands['dgrad'].append(('conv%d' % v, lambda v=v: KF.conv_fwd(dy.view(M, 1, 1, N), wt.view(K, 1, 1, N),
                                                                         (1, 1), (0, 0), None, v).view(M, K)))
        lib = _K.lib()
        for v in range(1, 10):
            if lib.conv_nhwc_wgrad_ring_ok(K, N, 1, 1, v):
                cands['wgrad'].append(('ring%d' % v, lambda v=v: KF.conv_wgrad(x.view(M, 1, 1, K), dy.view(M, 1, 1, N),
                                                                             (N, 1, 1, K), (1, 1), (0, 0), ring=v)))
        if hasattr(lib, 'gemm_nt'):
            from mxnet_maintenance_amd.ops import gemm as G
            for cfg in G.configs(M, N, K):
                cands['fwd'].append(('gemm%s' % (cfg,), lambda cfg=cfg: G.gemm_nt(x, w, cfg=cfg)))
            for cfg in G.configs(M, K, N):      # dX = dy . W: K output columns, reduction over N
                cands['dgrad'].append(('gemm%s' % (cfg,), lambda cfg=cfg: G.gemm_nt(dy, wt, cfg=cfg)))
        for kind, cl in cands.items():
            res = []
            for name, fn in cl:
                try:
                    out = fn()
                    if kind == 'fwd':
                        err = float((out.float() - ref_f).abs().max() / ref_f.abs().max())
                    elif kind == 'dgrad':
                        err = float((out.float() - ref_d).abs().max() / ref_d.abs().max())
                    else:
                        err = 0.0
                    t = timeit(fn, a.iters)
                    res.append((t, name, err))
                except Exception as e:  # noqa: BLE001
                    res.append((float('inf'), name + ' (%s)' % str(e)[:60], 0))
            res.sort()
            best = res[0]
            mm = next(r for r in res if r[1] == 'mm')
            tot.setdefault(kind, [0.0, 0.0])
            tot[kind][0] += mm[0]
            tot[kind][1] += best[0]
            print('%-5s M%d N%d K%d | mm %.1f us %.0f TF/s | best %s %.1f us %.0f TF/s (err %.1e)'
                  % (kind, M, N, K, mm[0] * 1e3, fl / mm[0] / 1e9, best[1], best[0] * 1e3, fl / best[0] / 1e9,
                     best[2]), flush=True)
            for t, name, err in res[:8]:
                print('      %-24s %.1f us %.0f TF/s err %.1e' % (name, t * 1e3, fl / t / 1e9, err))
            bad = [(name, err) for t, name, err in res if err > 2e-2]
            if bad:
                print('      WRONG RESULTS: %s' % bad, flush=True)
    for kind, (m, b) in tot.items():
        print('total %-5s mm %.1f us, best %.1f us' % (kind, m * 1e3, b * 1e3))


if __name__ == '__main__':
    main()
