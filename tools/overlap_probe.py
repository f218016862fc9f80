"""Copy/compute overlap probe for the engine's host -> device path.

Queues GEMM work on the compute stream, then uploads large host arrays with ``as_in_context``
(engine device ops on the copy stream).  Run under
``rocprofv3 --kernel-trace --memory-copy-trace --output-format csv`` and summarise with
tools/overlap_report.py: the H2D copies should overlap the GEMM kernels in time."""
import time

import numpy as np
import torch

import mxnet_maintenance_amd as mx


def main():
    dev = torch.device('cuda', 0)
    hosts = [mx.nd.array(np.random.rand(1 << 24).astype(np.float32)) for _ in range(4)]   # 64 MB each
    a = torch.randn(8192, 8192, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ups = []
    for i in range(4):
        for _ in range(6):
            a = torch.tanh(a @ a * 1e-4)
        ups.append(hosts[i].as_in_context(mx.gpu(0)))
    issue = time.perf_counter() - t0
    for u in ups:
        u.wait_to_read()
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
    ok = all(np.array_equal(u.asnumpy(), h.asnumpy()) for u, h in zip(ups, hosts))
    print('issued in %.1f ms, finished in %.1f ms, correct=%s' % (issue * 1e3, total * 1e3, ok))


if __name__ == '__main__':
    main()
