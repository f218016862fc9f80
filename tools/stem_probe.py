"""Stem (7x7/2, C=3 -> 64) forward and weight-gradient kernels at ResNet-50 b256, for counter runs:
    rocprofv3 --pmc <counters> --output-format csv -d <dir> -- python3 tools/stem_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from mxnet_maintenance_amd.ops import kernel_fns as KF  # noqa: E402

x = torch.randn(256, 224, 224, 3, device='cuda', dtype=torch.float16)
w = torch.randn(64, 7, 7, 3, device='cuda', dtype=torch.float16) * 0.1
dy = torch.randn(256, 112, 112, 64, device='cuda', dtype=torch.float16)
for _ in range(int(os.environ.get('REPS', '5'))):
    KF.conv_stem_fwd(x, w, (3, 3), bn_stats=True)
    KF.conv_stem_wgrad(x, dy, w.shape, (3, 3))
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, fn in (('fwd', lambda: KF.conv_stem_fwd(x, w, (3, 3), bn_stats=True)),
                 ('wgrad', lambda: KF.conv_stem_wgrad(x, dy, w.shape, (3, 3)))):
    s.record()
    for _ in range(10):
        fn()
    e.record()
    e.synchronize()
    print('stem %s %.3f ms' % (name, s.elapsed_time(e) / 10), flush=True)
