"""``/edit`` serving surface: a drop-in for the reference's ``server.py``.

Same HTTP contract as ``server.py``:
  * ``GET /`` (name, endpoints, status), ``GET /health``, ``POST /edit`` with
    ``EditRequest{image, prompt, steps, ref_image, blend_ratio, use_cfg}`` ->
    ``EditResponse{image, elapsed, status}`` (server.py:43-55, 162-230);
  * codec: base64 (optional ``data:...,`` prefix) -> PIL with EXIF transpose -> RGB,
    result -> JPEG q90 base64 (server.py:99-120);
  * request path: optional ``ref_image`` blend at 512x512 LANCZOS (server.py:205-209), input
    resized to 512x512 LANCZOS (server.py:131), fixed seed 42, ``use_cfg`` -> ``negative_prompt=""``
    (true CFG, server.py:135-153);
  * status codes: 503 model not loaded, 429 busy (one request at a time per GPU worker), 500
    ``str(e)`` (server.py:187-191, 226-230); one worker thread per GPU (server.py:39).

What differs is underneath: the pipeline is this package's HIP ``QwenImageEditPlusPipeline``
(loaded from local paths; no hub access), the codec is pluggable (``Codec``), and with
``workers > 1`` requests are spread over one process per GPU (``dispatch.GpuDispatcher``), so
the busy gate only answers 429 when every GPU is busy.

Run: ``python -m qwen_image_edit_streamdiffusion_amd.server`` (env ``QIE_MODEL_PATH``,
``QIE_LORA_PATH``, ``QIE_LORA_WEIGHT``, ``QIE_INT8``, ``QIE_ENCODERS=module:factory``,
``QIE_WORKERS``, ``QIE_REQUEST_TIMEOUT`` (seconds, multi-worker only), ``QIE_PORT`` = 8086).
"""
from __future__ import annotations

import asyncio
import base64
import importlib
import io
import os
import threading
import time
import traceback
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable, Optional

from PIL import Image, ImageOps
from pydantic import BaseModel

SERVE_SIZE = 512  # server.py:131, 207-208
SEED = 42         # server.py:139, 148
GUIDANCE = 3.5    # server.py:141, 150 (ignored by the model, forwarded like the reference)


class EditRequest(BaseModel):
    image: str
    prompt: str = "Transform into oil painting style"
    steps: int = 2
    ref_image: Optional[str] = None
    blend_ratio: float = 0.5
    use_cfg: bool = False


class EditResponse(BaseModel):
    image: str
    elapsed: float
    status: str


# ------------------------------------------------------------------------------------- codec
def base64_to_pil(b64_string: str) -> Image.Image:
    """server.py:99-112: strip a data-URL prefix, decode, EXIF-transpose, RGB."""
    if "," in b64_string:
        b64_string = b64_string.split(",", 1)[1]
    img = Image.open(io.BytesIO(base64.b64decode(b64_string)))
    img = ImageOps.exif_transpose(img)
    return img.convert("RGB")


def pil_to_base64(img: Image.Image, quality: int = 90) -> str:
    """server.py:115-119: JPEG quality 90, base64."""
    buf = io.BytesIO()
    img.save(buf, format="JPEG", quality=quality)
    return base64.b64encode(buf.getvalue()).decode()


@dataclass
class Codec:
    """Pluggable image codec (decode request images, encode the result)."""
    decode: Callable[[str], Image.Image] = base64_to_pil
    encode: Callable[[Image.Image], str] = pil_to_base64


# ----------------------------------------------------------------------------- request logic
def prepare_input(codec: Codec, req: EditRequest) -> Image.Image:
    """Decode and optionally blend with the reference image (server.py:201-209)."""
    img = codec.decode(req.image)
    if req.ref_image:
        ref = codec.decode(req.ref_image).resize((SERVE_SIZE, SERVE_SIZE), Image.LANCZOS)
        img = img.resize((SERVE_SIZE, SERVE_SIZE), Image.LANCZOS)
        img = Image.blend(img, ref, req.blend_ratio)
    return img


def process_image_sync(pipeline, image: Image.Image, prompt: str, steps: int, use_cfg: bool = False,
                       generator_device: Optional[str] = None) -> Image.Image:
    """server.py:122-158: 512x512 LANCZOS input, seed 42, negative_prompt="" iff use_cfg."""
    import torch
    image = image.resize((SERVE_SIZE, SERVE_SIZE), Image.LANCZOS)
    if generator_device is None:
        generator_device = "cuda" if torch.cuda.is_available() else "cpu"
    kw = dict(image=[image], prompt=prompt, num_inference_steps=steps, guidance_scale=GUIDANCE,
              generator=torch.Generator(device=generator_device).manual_seed(SEED))
    if use_cfg:
        kw["negative_prompt"] = ""
    with torch.no_grad():
        return pipeline(**kw).images[0]


class LocalWorker:
    """One pipeline in this process, one request at a time (server.py:39-40 executor + flag).

    Worker protocol (shared with ``dispatch.GpuDispatcher``): ``try_acquire() -> token | None``,
    ``run(token, image, request)`` on ``executor``, ``release(token)``."""

    size = 1

    def __init__(self, pipeline):
        self.pipeline = pipeline
        self._lock = threading.Lock()
        self.executor = ThreadPoolExecutor(max_workers=1)

    @property
    def loaded(self) -> bool:
        return self.pipeline is not None

    def try_acquire(self) -> Optional[int]:
        return 0 if self._lock.acquire(blocking=False) else None

    def release(self, token: int):
        self._lock.release()

    def run(self, token: int, image: Image.Image, req: EditRequest) -> Image.Image:
        return process_image_sync(self.pipeline, image, req.prompt, req.steps, req.use_cfg)


# ----------------------------------------------------------------------------------- loading
def _import(spec: str):
    mod, _, attr = spec.partition(":")
    return getattr(importlib.import_module(mod), attr)


def load_pipeline_from_env(device: str = "cuda"):
    """Local-path loader (the reference loads by hub name, server.py:58-79; no network here).

    ``QIE_MODEL_PATH``: diffusers snapshot or pre-quantised int8 image (weights.save_int8);
    ``QIE_LORA_PATH`` [+ ``QIE_LORA_WEIGHT``]: Lightning LoRA, fused at load;
    ``QIE_INT8=1``: quantise the linears (W8A8) after loading;
    ``QIE_ENCODERS=module:factory``: ``factory(pipeline)`` overrides ``prompt_encoder`` /
    ``image_encoder`` / ``latent_decoder``. By default the snapshot's own VAE (``vae/``) and
    Qwen2.5-VL prompt encoder (``text_encoder/`` + ``processor/``) run on the HIP path.
    """
    from .pipeline import QwenImageEditPlusPipeline
    path = os.environ.get("QIE_MODEL_PATH")
    if not path:
        raise RuntimeError("QIE_MODEL_PATH is not set (no hub downloads: point it at a local snapshot)")
    pipe = QwenImageEditPlusPipeline.from_pretrained(path, device=device)
    lora = os.environ.get("QIE_LORA_PATH")
    if lora:
        # raises (and so fails start-up) when the file's keys do not map onto the transformer
        n = pipe.load_lora_weights(lora, weight_name=os.environ.get("QIE_LORA_WEIGHT"))
        print(f"LoRA: fused {n} adapters from {lora}", flush=True)
    if os.environ.get("QIE_INT8") == "1" and not pipe.transformer.int8:
        pipe.transformer.quantize_int8()
    enc = os.environ.get("QIE_ENCODERS")
    if enc:
        _import(enc)(pipe)
    return pipe


def warmup(pipeline, runs: int = 2):
    """server.py:82-94: two gray 512x512 runs before serving."""
    dummy = Image.new("RGB", (SERVE_SIZE, SERVE_SIZE), color="gray")
    for _ in range(runs):
        process_image_sync(pipeline, dummy, "test", 2, False)


# ------------------------------------------------------------------------------------ the app
def create_app(loader: Optional[Callable[[], object]] = None, codec: Optional[Codec] = None,
               dispatcher=None, do_warmup: bool = True, title: str = "Qwen-Image-Edit API (MI355X HIP)"):
    """Build the FastAPI app.

    ``loader()`` returns a pipeline (default: ``load_pipeline_from_env``); a loader failure leaves
    the model unloaded and ``/edit`` answers 503, as the reference does before ``load_pipeline``
    has run. ``dispatcher``: a ``dispatch.GpuDispatcher`` serving requests from one process per
    GPU instead of an in-process pipeline.
    """
    from fastapi import FastAPI, HTTPException
    from fastapi.middleware.cors import CORSMiddleware

    import contextlib

    codec = codec or Codec()

    @contextlib.asynccontextmanager
    async def lifespan(app):
        _load()
        yield
        if dispatcher is not None:
            dispatcher.stop()

    app = FastAPI(title=title, lifespan=lifespan)
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True,
                       allow_methods=["*"], allow_headers=["*"])
    state = {"worker": None, "error": None}
    app.state.qie = state

    def _load():
        if dispatcher is not None:
            dispatcher.start()
            state["worker"] = dispatcher
            return
        try:
            pipe = (loader or load_pipeline_from_env)()
            if do_warmup:
                warmup(pipe)
            state["worker"] = LocalWorker(pipe)
        except Exception as e:  # keep serving: /edit -> 503, /health reports the error
            state["error"] = f"{type(e).__name__}: {e}"
            traceback.print_exc()

    @app.get("/")
    async def root():
        return {"name": "Qwen-Image-Edit-2509 API", "endpoints": ["/health", "/edit"], "status": "running"}

    @app.get("/health")
    async def health():
        w = state["worker"]
        out = {"status": "ok", "model_loaded": w is not None and w.loaded,
               "optimized": "MI355X HIP DiT (stream batch, batched CFG)"}
        if dispatcher is None:  # the dispatcher's parent process never initialises the GPU
            import torch
            out["gpu_memory"] = (f"{torch.cuda.max_memory_allocated() / 1e9:.2f} GB"
                                 if torch.cuda.is_available() else "N/A")
        else:
            out["workers"] = dispatcher.size
            out["worker_errors"] = dict(dispatcher.errors)
        if state["error"]:
            out["load_error"] = state["error"]
        return out

    @app.post("/edit", response_model=EditResponse)
    async def edit_image(request: EditRequest):
        w = state["worker"]
        if w is None or not w.loaded:
            raise HTTPException(status_code=503, detail="Model not loaded")
        token = w.try_acquire()
        if token is None:
            raise HTTPException(status_code=429, detail="Server is busy processing another request")
        try:
            start = time.time()
            image = prepare_input(codec, request)
            loop = asyncio.get_event_loop()
            result = await loop.run_in_executor(w.executor, w.run, token, image, request)
            return EditResponse(image=codec.encode(result), elapsed=time.time() - start, status="success")
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))
        finally:
            w.release(token)

    return app


def main():
    import uvicorn
    n = int(os.environ.get("QIE_WORKERS", "1"))
    dispatcher = None
    if n > 1:
        from .dispatch import GpuDispatcher
        rt = os.environ.get("QIE_REQUEST_TIMEOUT")  # seconds; a worker silent for longer is replaced
        dispatcher = GpuDispatcher(n, "qwen_image_edit_streamdiffusion_amd.server:load_pipeline_from_env",
                                   request_timeout=float(rt) if rt else None)
    app = create_app(dispatcher=dispatcher)
    uvicorn.run(app, host=os.environ.get("QIE_HOST", "0.0.0.0"), port=int(os.environ.get("QIE_PORT", "8086")))


if __name__ == "__main__":
    main()
