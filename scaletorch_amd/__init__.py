"""scaletorch_amd -- an MI355X-native (gfx950 / CDNA4) 5-D parallel LLM training framework.

PyTorch-ROCm for orchestration, hand-written HIP kernels (csrc/) for the hot
ops, RCCL over xGMI for communication.  Capability parity target:
jianzhnie/ScaleTorch.
"""
__version__ = "0.1.0"
