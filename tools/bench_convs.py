"""Per-layer conv timing for ResNet-50 v1b at batch 256, NHWC fp16 on one MI355X.

Compares the MIOpen path (torch conv on channels_last views) with the plain
GEMM path (hipBLASLt via torch.mm) for 1x1 convolutions, and with the
in-tree HIP implicit-GEMM kernels when they are built.  Output: one line per
layer shape with fwd / dgrad / wgrad milliseconds, and per-step totals.
"""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

# (H_in, Cin, Cout, k, stride, count) for ResNet-50 v1b (stride on the 3x3)
LAYERS = [
    (224, 3, 64, 7, 2, 1),
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (28, 128, 512, 1, 1, 4), (56, 256, 512, 1, 2, 1),
    (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (14, 256, 1024, 1, 1, 6), (28, 512, 1024, 1, 2, 1),
    (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (7, 512, 2048, 1, 1, 3), (14, 1024, 2048, 1, 2, 1),
    (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--dtype', default='float16')
    ap.add_argument('--hip', action='store_true', help='also time the in-tree HIP conv kernels')
    args = ap.parse_args()
    dt = getattr(torch, args.dtype)
    dev = 'cuda'
    N = args.batch
    hipk = None
    if args.hip:
        sys.path.insert(0, '.')
        from mxnet_maintenance_amd.ops import kernel_fns as hipk  # noqa: F811
    tot = {'miopen': [0, 0, 0], 'mm': [0, 0, 0], 'hip': [0, 0, 0]}
    rows = []
    for (H, Cin, Cout, k, s, cnt) in LAYERS:
        pad = k // 2
        Ho = (H + 2 * pad - k) // s + 1
        x = torch.randn(N, H, H, Cin, device=dev, dtype=dt)
        w = torch.randn(Cout, k, k, Cin, device=dev, dtype=dt) * 0.05
        dy = torch.randn(N, Ho, Ho, Cout, device=dev, dtype=dt)
        xc = x.permute(0, 3, 1, 2)
        wc = w.permute(0, 3, 1, 2)
        dyc = dy.permute(0, 3, 1, 2)
        flops = 2.0 * N * Ho * Ho * Cout * Cin * k * k
        r = {'shape': [H, Cin, Cout, k, s], 'count': cnt, 'gflop': flops / 1e9}
        f = timeit(lambda: F.conv2d(xc, wc, None, s, pad))
        bd = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [pad, pad], [1, 1],
                                                                False, [0, 0], 1, [True, False, False]))
        bw = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [s, s], [pad, pad], [1, 1],
                                                                False, [0, 0], 1, [False, True, False]))
        r['miopen'] = [f, bd, bw]
        for i, v in enumerate((f, bd, bw)):
            tot['miopen'][i] += v * cnt
        if k == 1:
            w2 = w.reshape(Cout, Cin)
            if s == 1:
                x2 = x.reshape(-1, Cin)
                dy2 = dy.reshape(-1, Cout)
                f2 = timeit(lambda: torch.mm(x2, w2.t()))
                bd2 = timeit(lambda: torch.mm(dy2, w2))
                bw2 = timeit(lambda: torch.mm(dy2.t(), x2))
            else:
                dy2 = dy.reshape(-1, Cout)
                f2 = timeit(lambda: torch.mm(x[:, ::s, ::s].reshape(-1, Cin), w2.t()))

                def dgrad():
                    dx = torch.zeros_like(x)
                    dx[:, ::s, ::s] = torch.mm(dy2, w2).view(N, Ho, Ho, Cin)
                    return dx
                bd2 = timeit(dgrad)
                bw2 = timeit(lambda: torch.mm(dy2.t(), x[:, ::s, ::s].reshape(-1, Cin)))
            r['mm'] = [f2, bd2, bw2]
        else:
            r['mm'] = r['miopen']
        for i, v in enumerate(r['mm']):
            tot['mm'][i] += v * cnt
        if hipk is not None and hipk.conv_ok_shape(x, w, (s, s), (pad, pad)):
            hf = timeit(lambda: hipk.conv_fwd(x, w, (s, s), (pad, pad)))
            r['hip_fwd'] = hf
            yref = F.conv2d(xc, wc, None, s, pad).permute(0, 2, 3, 1).float()
            yh = hipk.conv_fwd(x, w, (s, s), (pad, pad)).float()
            r['hip_err'] = float((yh - yref).abs().max() / (yref.abs().max() + 1e-6))
            r['hip_tflops'] = flops / hf / 1e9
        r['miopen_tflops'] = [flops / t / 1e9 for t in r['miopen']]
        rows.append(r)
        print(json.dumps(r), flush=True)
        del x, w, dy
    print(json.dumps({'total_ms_per_step': tot}), flush=True)


if __name__ == '__main__':
    main()
