"""Where does the bf16 deformable-conv offset gradient differ from fp32?  Runs the test's cases three
ways on the same bf16-rounded inputs: CPU fp32 reference, GPU kernels in fp32, GPU kernels in bf16,
and prints the relative-norm differences of every output/gradient pair."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import test_deform_conv as T  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-12))


def main():
    for case in T.CASES:
        x, off, mask, w = T._inputs(case)
        dev16 = [t.to('cuda', torch.bfloat16) if t is not None else None for t in (x, off, mask, w)]
        base = [t.float().cpu() if t is not None else None for t in dev16]
        ref = T._run(case, *(t.clone() if t is not None else None for t in base), grad_dtype=torch.bfloat16)
        g32 = T._run(case, *(t.cuda() if t is not None else None for t in base), grad_dtype=torch.bfloat16)
        g16 = T._run(case, *dev16, grad_dtype=torch.bfloat16)
        names = ['out', 'dx', 'doffset'] + (['dmask'] if mask is not None else []) + ['dweight']
        for n, r, a, b in zip(names, ref, g32, g16):
            print('case %s %-8s gpu32-vs-ref %.2e  gpu16-vs-ref %.2e  gpu16-vs-gpu32 %.2e  |ref| %.3e'
                  % (case[:4], n, rel(a, r), rel(b, r), rel(b, a), float(r.norm())), flush=True)


if __name__ == '__main__':
    main()
