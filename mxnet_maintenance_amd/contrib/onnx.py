"""ONNX model import / export (reference python/mxnet/contrib/onnx/__init__.py): the importer and the
exporter live in ``mxnet_maintenance_amd.onnx``; this is the contrib path the reference keeps."""
from ..onnx import import_model, get_model_metadata, import_to_gluon, export_model  # noqa: F401

__all__ = ['import_model', 'get_model_metadata', 'import_to_gluon', 'export_model']
