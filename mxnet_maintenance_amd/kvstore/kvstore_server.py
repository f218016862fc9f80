"""Server role (parity: python/mxnet/kvstore/kvstore_server.py).

With RCCL all-reduce there are no parameter servers; a process started with
DMLC_ROLE=server/scheduler simply exits after reporting that, so legacy
launch scripts keep working.
"""
import logging
import os


class KVStoreServer:
    def __init__(self, kvstore):
        self.kvstore = kvstore

    def run(self):
        logging.info('KVStoreServer: no parameter servers are needed (RCCL all-reduce); exiting.')


def _init_kvstore_server_module():
    role = os.environ.get('DMLC_ROLE', 'worker')
    if role in ('server', 'scheduler'):
        KVStoreServer(None).run()
