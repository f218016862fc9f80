"""Environment knobs: one typed registry for every variable the framework reads.

Parity: docs/static_site/src/pages/api/faq/env_var.md in the reference.  MXNet
names are kept where the concept carries over (engine type, worker threads,
autotune, update-on-kvstore, MXNET_HOME); MI355X-specific knobs use the
``MXAMD_`` prefix.  ``describe()`` prints the table; ``get(name)`` returns the
typed value (environment first, then the default).
"""
import os

__all__ = ['KNOBS', 'get', 'describe']

# name: (type, default, meaning, reference knob it replaces or '')
KNOBS = {
    'MXNET_ENGINE_TYPE': (str, 'ThreadedEnginePerDevice', 'host dependency engine: NaiveEngine (synchronous, '
                          'debugging), ThreadedEngine, ThreadedEnginePerDevice', 'MXNET_ENGINE_TYPE'),
    'MXNET_CPU_WORKER_NTHREADS': (int, 4, 'native engine worker threads (IO, host copies, kvstore host work)',
                                  'MXNET_CPU_WORKER_NTHREADS'),
    'MXNET_CUDNN_AUTOTUNE_DEFAULT': (int, 1, 'conv algorithm autotuning (HIP implicit-GEMM / hipBLASLt / MIOpen / '
                                     'split-K wgrad timed per shape); 0 = heuristic choice',
                                     'MXNET_CUDNN_AUTOTUNE_DEFAULT'),
    'MXNET_ENFORCE_DETERMINISM': (int, 0, 'bitwise-reproducible training: the autotuner only admits kernels with a '
                                  'fixed reduction order (the in-tree MFMA kernels, no vendor split-K / atomic '
                                  'candidates), atomic accumulations switch to ordered reductions, and torch / MIOpen '
                                  'run their deterministic algorithms', 'MXNET_ENFORCE_DETERMINISM'),
    'MXNET_UPDATE_ON_KVSTORE': (int, 1, 'Module/model API: run the optimizer inside the kvstore',
                                'MXNET_UPDATE_ON_KVSTORE'),
    'MXNET_HOME': (str, os.path.join(os.path.expanduser('~'), '.mxnet'), 'dataset / model cache root', 'MXNET_HOME'),
    'MXNET_GLUON_REPO': (str, 'https://apache-mxnet.s3-accelerate.dualstack.amazonaws.com/',
                         'model/dataset repository URL (unused offline)', 'MXNET_GLUON_REPO'),
    'MXNET_TEST_DEVICE': (str, 'cpu', 'test_utils.default_context(): cpu or gpu', ''),
    'MXAMD_BUCKET_MB': (float, 0.0, 'gradient bucket size for the overlapped RCCL all-reduce (MiB); default (0): '
                        'a quarter of the gradient bytes clamped to [16, 64] MiB (parallel/buckets.py cost model '
                        'for 7-link xGMI rings)',
                        'MXNET_KVSTORE_BIGARRAY_BOUND'),
    'MXAMD_TAIL_BUCKET_MB': (float, 4.0, 'bucket cap for the gradients of the first layers (the last to be produced '
                             'in backward): their all-reduce cannot overlap compute, so smaller buckets shorten the '
                             'exposed tail', ''),
    'MXAMD_FLAT_ARENA': (int, 1, 'Trainer keeps params/grads in flat per-dtype arenas (one fused optimizer kernel, '
                         'zero-copy all-reduce buckets)', ''),
    'MXAMD_DIST_BACKEND': (str, '', 'force torch.distributed backend (gloo for CPU runs); default nccl(=RCCL) on GPU',
                           ''),
    'MXAMD_VENDOR_MARGIN': (float, 0.05, 'autotuner: a MIOpen / hipBLASLt candidate must beat the fastest in-tree '
                            'kernel by this fraction to be chosen (near-ties within timing noise go in-tree)', ''),
    'MXAMD_DISABLE_HIP': (int, 0, 'do not load the gfx950 HIP kernel extension (debug only)', ''),
    'MXAMD_ALLOW_TORCH_FALLBACK': (int, 0, 'allow silent torch fallbacks when the HIP extension is missing on a GPU',
                                   ''),
    'MXAMD_CONV_HIP': (int, 1, 'offer the HIP implicit-GEMM conv kernels to the autotuner', ''),
    'MXAMD_PROFILER_SYNC': (int, 0, 'profiler synchronises the device around each op span (true GPU op time)', ''),
    'MXAMD_OFFLOAD_ARCH': (str, 'gfx950', 'rtc / extension build target', ''),
    'MXAMD_RTC_CACHE': (str, os.path.expanduser('~/.cache/mxamd_rtc'), 'code-object cache for mx.rtc kernels', ''),
}


def get(name, default=None):
    typ, dflt, _, _ = KNOBS.get(name, (str, default, '', ''))
    v = os.environ.get(name)
    if v is None or v == '':
        return dflt if default is None else default
    try:
        return typ(float(v)) if typ is int else typ(v)
    except ValueError:
        return v


def describe():
    rows = ['%-30s %-8s %-30s %s' % ('name', 'type', 'default', 'meaning')]
    for k, (t, d, doc, ref) in sorted(KNOBS.items()):
        rows.append('%-30s %-8s %-30s %s%s' % (k, t.__name__, str(d)[:30], doc,
                                              (' [reference: %s]' % ref) if ref and ref != k else ''))
    return '\n'.join(rows)
