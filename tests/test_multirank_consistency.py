"""Multi-rank readiness on CPU (gloo, 2 processes): autotuning picks the SAME kernel on every rank,
and a HIP-graph capture failure on one rank makes every rank fall back to eager together."""
import os
import socket

import torch.multiprocessing as tmp


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, which):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'MASTER_ADDR': '127.0.0.1',
                       'MASTER_PORT': str(port), 'MXAMD_DIST_BACKEND': 'gloo', 'LOCAL_RANK': str(rank)})
    import time
    from mxnet_maintenance_amd.parallel import dist
    try:
        dist.init()
        if which == 'autotune':
            from mxnet_maintenance_amd.ops import kernel_fns as KF
            # rank 0 measures A fast, rank 1 measures B fast: without agreement they would diverge.
            # The per-rank times are injected (no sleeps), so host load cannot change the outcome.
            delay = {0: {'candA': 1.0, 'candB': 5.0}, 1: {'candA': 10.0, 'candB': 4.0}}[rank]

            def fake_measure(fn, reps):
                r = fn()
                return delay[r] * reps, r
            KF._measure = fake_measure

            def mk(name):
                return lambda: name
            best, out = KF._time_candidates([('candA', mk('candA')), ('candB', mk('candB'))], reps=1,
                                            key=('test', rank))
            q.put((rank, best, out))
        else:
            from mxnet_maintenance_amd.gluon import graph_step as GS
            calls = []

            def step():
                calls.append('eager')
                return len(calls)
            g = GS.GraphStep(step, None, warmup=1, fallback=True)

            class FakeGraph:
                def replay(self):
                    calls.append('replay')

            def capture(inputs):
                if rank == 0:
                    raise RuntimeError('forced capture failure')
                g._graph = FakeGraph()
                g._rng = None
            g._capture = capture
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter('ignore')
                for _ in range(3):
                    g()
            q.put((rank, g._eager_only, g.captured, calls))
    except Exception:
        import traceback
        q.put((rank, 'ERR', traceback.format_exc(), None))
    finally:
        import torch.distributed as tdist
        if tdist.is_initialized():
            tdist.destroy_process_group()


def _run(which):
    ctx = tmp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, which)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        item = q.get(timeout=240)
        res[item[0]] = item
    for p in ps:
        p.join(timeout=60)
    for r in range(2):
        assert res[r][1] != 'ERR', res[r][2]
    return res


def test_autotune_choice_identical_on_every_rank():
    res = _run('autotune')
    assert res[0][1] == res[1][1] == 'candB'       # max over ranks: A 10 ms, B 5 ms
    assert res[0][2] == res[1][2] == 'candB'


def test_graph_capture_failure_on_one_rank_makes_all_ranks_eager():
    res = _run('graph')
    for r in range(2):
        _, eager_only, captured, calls = res[r]
        assert eager_only and not captured
        assert calls == ['eager', 'eager', 'eager'], calls      # no rank replayed a graph
