"""MI355X-native (gfx950) Qwen-Image-Edit-2509 denoise hot path.

Drop-in for the reference's hot path (shi3z/Qwen-Image-Edit-StreamDiffusion):
the diffusers ``QwenImageTransformer2DModel`` module surface, the
``QwenImageEditPlusPipeline`` call surface with batched CFG, and the
qwen_realtime stream-batch loop -- all arithmetic in hand-written HIP kernels
(libqie.so, include/qie.h) loaded through a thin C ABI.
"""
from ._lib import QieError, load as load_library
from .transformer import QwenImageTransformer2DModel, TransformerConfig
from .scheduler import FlowMatchEulerDiscreteScheduler, calculate_shift
from .pipeline import QwenImageEditPlusPipeline, calculate_dimensions
from .stream import StreamConfig, CachedConditions, StreamBatchDenoiser, QwenRealtimePipeline

__all__ = [
    "QieError", "load_library", "QwenImageTransformer2DModel", "TransformerConfig",
    "FlowMatchEulerDiscreteScheduler", "calculate_shift", "QwenImageEditPlusPipeline",
    "calculate_dimensions", "StreamConfig", "CachedConditions", "StreamBatchDenoiser",
    "QwenRealtimePipeline",
]
