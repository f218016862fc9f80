"""Host cost per imperative GPU operator on the caller's stream (MXNET_GPU_WORKER_NTHREADS=1) and
through the native engine's worker-stream dispatcher (2 / 4 slots), plus the two-chain wall time of
tools/worker_streams_probe.py's spin operators (independent chains overlap on 2+ slots).

    python tools/dispatch_overhead_probe.py [--ops 4000]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def per_op_us(workers, n):
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import engine
    engine.set_gpu_workers(workers)
    ctx = mx.gpu(0)
    a = mx.nd.ones((16, 16), ctx=ctx)
    b = mx.nd.ones((16, 16), ctx=ctx)
    for _ in range(50):
        a = mx.nd.relu(a)
    mx.nd.waitall()
    t0 = time.perf_counter()
    for i in range(n // 2):
        a = mx.nd.relu(a)           # two independent chains
        b = mx.nd.relu(b)
    t1 = time.perf_counter()
    mx.nd.waitall()
    return (t1 - t0) / n * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ops', type=int, default=4000)
    a = ap.parse_args()
    import worker_streams_probe as W
    out = {}
    for w in (1, 2, 4):
        out['host_us_per_op_workers%d' % w] = round(per_op_us(w, a.ops), 2)
    for w in (1, 2):
        W.run(w, 2, 2_000_000)            # warm-up (operator registration, stream creation)
        ms, ok = W.run(w, 20, 2_000_000)
        out['two_spin_chains_ms_workers%d' % w] = round(ms, 1)
        out['two_spin_chains_ok_workers%d' % w] = ok
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
