"""ONNX export (``mx.onnx``) and import (``mx.contrib.onnx``).

Reference: python/mxnet/onnx/__init__.py (export_model, get_operator_support) and
python/mxnet/contrib/onnx/__init__.py (import_model, get_model_metadata, import_to_gluon).  The
ONNX protobuf schema is declared in ``_proto`` (the onnx wheel is not installed).
"""
from .mx2onnx import export_model, get_operator_support
from .onnx2mx import import_model, get_model_metadata, import_to_gluon
from ._proto import load_model

__all__ = ['export_model', 'get_operator_support', 'import_model', 'get_model_metadata', 'import_to_gluon',
           'load_model']
