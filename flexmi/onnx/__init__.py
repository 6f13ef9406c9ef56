"""flexmi.onnx -- ONNX frontend (``python/flexflow/onnx``) with a built-in protobuf wire codec (the
``onnx`` package is not required)."""
from .model import ONNXModel  # noqa: F401
from .proto import decode_model, encode_model, encode_node  # noqa: F401
