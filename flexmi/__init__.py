"""flexmi -- an MI355X-native auto-parallelizing training framework with the capabilities of
FlexFlow / DLRM-FlexFlow (SOAP parallelization search, strategy files, model-builder API),
built on PyTorch-ROCm buffers, hand-written CDNA4 HIP kernels and RCCL over xGMI.

This package is the ``dlrm-flexflow_amd`` framework: ``flexmi.core`` (FFConfig/FFModel API),
``flexmi.ops`` (operators + HIP kernel bindings), ``flexmi.parallel`` (sharding algebra,
strategies, simulator, MCMC search, RCCL comm), ``flexmi.models`` (DLRM, CNNs, NMT),
``flexmi.runtime`` (plan compiler/executor), ``flexmi.utils``, frontends ``flexmi.keras``,
``flexmi.torch``, ``flexmi.onnx``.
"""
__version__ = "0.1.0"
