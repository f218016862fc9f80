"""Server role of the ``dist_async`` parameter server.

Parity: python/mxnet/kvstore/kvstore_server.py (``KVStoreServer`` + ``_init_kvstore_server_module``,
started when a process runs with ``DMLC_ROLE=server``).

Synchronous data parallelism here is RCCL all-reduce (no servers).  The asynchronous store
(``kvstore/dist_async.py``) does have a server: by default rank 0's worker process hosts it; with
``DMLC_NUM_SERVER=1`` a separate process started with ``DMLC_ROLE=server`` hosts it instead.  That
process joins the RPC world as rank ``DMLC_NUM_WORKER`` (named ``server``), serves init / push / pull /
set_optimizer / barrier requests on its RPC threads, and exits once every worker has shut down.
A ``scheduler`` role has nothing to coordinate (the RPC rendezvous is the TCP store at MASTER_ADDR) and
returns immediately.
"""
import logging
import os


class KVStoreServer:
    """Hosts the dist_async store in this process until all workers are done."""

    def __init__(self, kvstore=None):
        self.kvstore = kvstore

    def run(self):
        role = os.environ.get('DMLC_ROLE', 'server')
        if role == 'scheduler':
            logging.info('KVStoreServer: no scheduler is needed (RPC rendezvous at MASTER_ADDR); exiting.')
            return
        from . import dist_async
        if not dist_async.dedicated_server():
            raise RuntimeError('KVStoreServer: a server process needs DMLC_NUM_SERVER >= 1 so the workers '
                               'address it instead of rank 0')
        nworkers = int(os.environ.get('DMLC_NUM_WORKER', os.environ.get('WORLD_SIZE', '1')))
        dist_async._init_rpc(nworkers, nworkers, name='server')
        logging.info('KVStoreServer: serving %d dist_async workers', nworkers)
        # a graceful shutdown blocks until every worker has called shutdown (i.e. finished training)
        dist_async._shutdown_rpc()


_CHILD_ENV = 'MXAMD_KVSTORE_SERVER_CHILD'


def _init_kvstore_server_module():
    """Entry for ``DMLC_ROLE=server`` / ``scheduler`` processes at ``import``: serve, then return True
    so the caller exits (the reference does this from ``import mxnet``).

    Serving cannot happen inside the package import itself: the RPC threads unpickle the server
    functions by importing this package, whose import lock the importing thread still holds.  So the
    importing process runs the server in a child python that imports the package first and serves
    after and exits with its status."""
    role = os.environ.get('DMLC_ROLE', 'worker')
    if role not in ('server', 'scheduler') or os.environ.get(_CHILD_ENV):
        return False
    import subprocess
    import sys
    env = dict(os.environ)
    env[_CHILD_ENV] = '1'
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env['PYTHONPATH'] = root + (os.pathsep + env['PYTHONPATH'] if env.get('PYTHONPATH') else '')
    rc = subprocess.call([sys.executable, '-c', 'import logging; logging.basicConfig(level=logging.INFO); '
                          'from mxnet_maintenance_amd.kvstore.kvstore_server import KVStoreServer; '
                          'KVStoreServer(None).run()'], env=env)
    if rc != 0:
        raise SystemExit(rc)
    return True


if __name__ == '__main__':
    logging.basicConfig(level=logging.INFO)
    KVStoreServer(None).run()
