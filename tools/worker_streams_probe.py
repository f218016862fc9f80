"""Two independent imperative chains with MXNET_GPU_WORKER_NTHREADS=2 (engine.op_stream): run under
``rocprofv3 --kernel-trace`` and summarise with ``--report DIR`` to see the two chains' kernels on two
streams overlapping in time.  Each operator is a Custom op whose body is a long single-workgroup spin
kernel, so one stream alone leaves the GPU idle and two chains should take about half the time."""
import argparse
import csv
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_REGISTERED = []


def _spin_op(cycles):
    """A Custom operator whose body is one single-workgroup spin kernel (torch.cuda._sleep) followed
    by a copy: long GPU work per dispatch that occupies one CU, so one stream leaves the GPU idle."""
    import torch
    import mxnet_maintenance_amd as mx
    if _REGISTERED:
        return

    class Spin(mx.operator.CustomOp):
        def forward(self, is_train, req, in_data, out_data, aux):
            torch.cuda._sleep(cycles)
            self.assign(out_data[0], req[0], in_data[0] + 1)

    @mx.operator.register('spin_probe')
    class SpinProp(mx.operator.CustomOpProp):
        def create_operator(self, ctx, shapes, dtypes):
            return Spin()
    _REGISTERED.append(True)


def run(workers, n, cycles):
    import numpy as onp
    import mxnet_maintenance_amd as mx
    from mxnet_maintenance_amd import engine
    _spin_op(cycles)
    engine.set_gpu_workers(workers)
    ctx = mx.gpu(0)
    x1 = mx.nd.zeros((64, 64), ctx=ctx)
    x2 = mx.nd.zeros((64, 64), ctx=ctx)
    mx.nd.waitall()
    t0 = time.time()
    a, b = x1, x2
    for _ in range(n):
        a = mx.nd.Custom(a, op_type='spin_probe')
        b = mx.nd.Custom(b, op_type='spin_probe')
    ok = float(a.asnumpy()[0, 0]) == n and float(b.asnumpy()[0, 0]) == n
    mx.nd.waitall()
    return (time.time() - t0) * 1e3, ok


def report(d):
    rows = []
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        sid = r.get('Stream_Id') or r.get('Queue_Id')
        by.setdefault(sid, []).append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    print('kernels per stream/queue:', {k: len(v) for k, v in by.items()})
    keys = [k for k, v in by.items() if len(v) > 10]
    if len(keys) >= 2:
        a, b = sorted(by[keys[0]]), sorted(by[keys[1]])
        ov = 0
        j = 0
        for s, e in a:
            while j < len(b) and b[j][1] < s:
                j += 1
            k = j
            while k < len(b) and b[k][0] < e:
                ov += min(e, b[k][1]) - max(s, b[k][0])
                k += 1
        busy = sum(e - s for s, e in a)
        print('overlapped kernel time: %.3f ms of %.3f ms on the first stream (%.0f%%)'
              % (ov / 1e6, busy / 1e6, 100.0 * ov / max(1, busy)))


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--workers', type=int, default=2)
    ap.add_argument('--n', type=int, default=20)
    ap.add_argument('--cycles', type=int, default=2000000)
    ap.add_argument('--report', default=None)
    args = ap.parse_args()
    if args.report:
        report(args.report)
    else:
        run(args.workers, 2, args.cycles)
        ms, ok = run(args.workers, args.n, args.cycles)
        print('workers=%d: %.2f ms for 2 independent chains x %d spin ops (results %s)'
              % (args.workers, ms, args.n, 'ok' if ok else 'WRONG'))
