"""MI355X-native (gfx950) Qwen-Image-Edit-2509 denoise hot path.

Drop-in for the reference's hot path (shi3z/Qwen-Image-Edit-StreamDiffusion):
the diffusers ``QwenImageTransformer2DModel`` module surface, the
``QwenImageEditPlusPipeline`` call surface with batched CFG, and the
qwen_realtime stream-batch loop -- all arithmetic in hand-written HIP kernels
(libqie.so, include/qie.h) loaded through a thin C ABI.
"""
import os as _os

# The transformer overlaps its text stream with the image stream on a second HIP stream; once RCCL
# adds its own streams (parallel.py), HIP's default 4 hardware queues per process make the two
# model streams share a queue and the overlap serialises (~9 % per step). Effective only when this
# package is imported before HIP initialises; parallel.init_distributed warns otherwise.
if int(_os.environ.get("GPU_MAX_HW_QUEUES") or 0) < 8:  # raise an inherited 4, keep a larger value
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"

from ._lib import QieError, load as load_library  # noqa: E402
from .transformer import QwenImageTransformer2DModel, TransformerConfig  # noqa: E402
from .scheduler import FlowMatchEulerDiscreteScheduler, calculate_shift  # noqa: E402
from .pipeline import QwenImageEditPlusPipeline, calculate_dimensions  # noqa: E402
from .stream import StreamConfig, CachedConditions, StreamBatchDenoiser, QwenRealtimePipeline  # noqa: E402

__all__ = [
    "QieError", "load_library", "QwenImageTransformer2DModel", "TransformerConfig",
    "FlowMatchEulerDiscreteScheduler", "calculate_shift", "QwenImageEditPlusPipeline",
    "calculate_dimensions", "StreamConfig", "CachedConditions", "StreamBatchDenoiser",
    "QwenRealtimePipeline",
]
