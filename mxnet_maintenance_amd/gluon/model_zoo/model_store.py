"""Pretrained model store (parity: python/mxnet/gluon/model_zoo/model_store.py).

This host has no network access; ``get_model_file`` returns a locally cached
``<root>/<name>-<hash>.params`` if present and raises otherwise.
"""
import glob
import os

__all__ = ['get_model_file', 'purge']


def get_model_file(name, root=os.path.join('~', '.mxnet', 'models')):
    """Path of ``name``'s pretrained ``.params``: looked up in ``root``, then in the local model
    caches ($MXNET_HOME/models, ~/.mxnet/models).  There is no network download."""
    roots = [os.path.expanduser(root)]
    if os.environ.get('MXNET_HOME'):
        roots.append(os.path.join(os.environ['MXNET_HOME'], 'models'))
    roots.append(os.path.expanduser(os.path.join('~', '.mxnet', 'models')))
    for r in roots:
        cands = sorted(glob.glob(os.path.join(r, name + '-*.params')))
        if cands:
            return cands[0]
    raise RuntimeError('Pretrained weights for %s are not available offline (looked in %s)' % (name, roots))


def purge(root=os.path.join('~', '.mxnet', 'models')):
    root = os.path.expanduser(root)
    for f in glob.glob(os.path.join(root, '*.params')):
        os.remove(f)
