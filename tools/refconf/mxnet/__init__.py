"""Process-level ``mxnet`` alias for worker processes of the reference tests (forkserver / spawn
children do not load the pytest plugin): importing ``mxnet`` installs the alias finder and replaces
this module with ``mxnet_maintenance_amd``."""
import sys

import mxalias  # noqa: F401  (installs the mxnet.* -> mxnet_maintenance_amd.* finder)
import mxnet_maintenance_amd as _framework

sys.modules[__name__] = _framework
