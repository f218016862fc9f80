"""GraphStep vs eager on a hybridized NHWC fp16 ResNet: per-parameter relative error of a graph run
and of a second eager run against a first eager run (the second eager run measures the run-to-run
noise of fp16 training with nondeterministic vendor kernels).

    python tools/debug_graph_vs_eager.py [resnet18_v1|resnet50_v1b] [steps]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from test_resnet_gpu import _train  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'resnet18_v1'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    le, we, names = _train(False, steps=steps, name=name, with_names=True)
    le2, we2, _ = _train(False, steps=steps, name=name, with_names=True)
    lg, wg, _ = _train(True, steps=steps, name=name, with_names=True)
    print('loss eager ', np.round(le, 4))
    print('loss eager2', np.round(le2, 4))
    print('loss graph ', np.round(lg, 4))
    worst = []
    for n, a, b, g in zip(names, we, we2, wg):
        d = np.linalg.norm(a) + 1e-6
        e2 = np.linalg.norm(b - a) / d
        eg = np.linalg.norm(g - a) / d
        worst.append((eg, e2, n))
        print('%-60s eager2 %.2e  graph %.2e %s' % (n, e2, eg, '<<' if eg > 3 * e2 + 1e-4 else ''))
    worst.sort(reverse=True)
    print('worst graph errors:', worst[:5])


if __name__ == '__main__':
    main()
