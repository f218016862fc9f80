"""Pretrained model store (parity: python/mxnet/gluon/model_zoo/model_store.py).

This host has no network access; ``get_model_file`` returns a locally cached
``<root>/<name>-<hash>.params`` if present and raises otherwise.
"""
import glob
import os

__all__ = ['get_model_file', 'purge']


def get_model_file(name, root=os.path.join('~', '.mxnet', 'models')):
    root = os.path.expanduser(root)
    cands = sorted(glob.glob(os.path.join(root, name + '*.params')))
    if cands:
        return cands[0]
    raise RuntimeError('Pretrained weights for %s are not available offline (looked in %s)' % (name, root))


def purge(root=os.path.join('~', '.mxnet', 'models')):
    root = os.path.expanduser(root)
    for f in glob.glob(os.path.join(root, '*.params')):
        os.remove(f)
