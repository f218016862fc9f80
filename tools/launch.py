#!/usr/bin/env python
"""Launch a data-parallel job on this node: one worker process per GPU.

Parity: reference ``tools/launch.py:57`` (``-n`` workers, ``--launcher local``).
There are no parameter servers here (KVStore dist_* types run over a
torch.distributed process group), so ``-s`` is accepted and ignored.

    python tools/launch.py -n 8 python train.py --kv-store device

Exit status: 0 if all workers succeed, else the first failing worker's code.
"""
import argparse
import os
import sys


def _load_launch():
    """parallel/launch.py loaded by file path: importing the package would import torch and the HIP
    extensions into this launcher parent, which must stay GPU-free (its children are the GPU ranks)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'mxnet_maintenance_amd',
                        'parallel', 'launch.py')
    spec = importlib.util.spec_from_file_location('_mxamd_launch', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.launch


def main():
    ap = argparse.ArgumentParser(description='Launch a local multi-process (one per GPU) job')
    ap.add_argument('-n', '--num-workers', type=int, required=True)
    ap.add_argument('-s', '--num-servers', type=int, default=0, help='ignored (no parameter servers)')
    ap.add_argument('--launcher', default='local', choices=['local'])
    ap.add_argument('--master-addr', default='127.0.0.1')
    ap.add_argument('--master-port', type=int, default=None)
    ap.add_argument('--timeout', type=float, default=None, help='kill the job after this many seconds')
    ap.add_argument('command', nargs=argparse.REMAINDER)
    args = ap.parse_args()
    if not args.command:
        ap.error('no command given')
    launch = _load_launch()
    sys.exit(launch(args.command, args.num_workers, master_addr=args.master_addr,
                    master_port=args.master_port, timeout=args.timeout))


if __name__ == '__main__':
    main()
