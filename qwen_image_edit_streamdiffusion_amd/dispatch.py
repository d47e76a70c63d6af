"""Multi-GPU request dispatcher for the ``/edit`` server.

The reference serves one request at a time on one pinned GPU (``CUDA_VISIBLE_DEVICES='7'``,
one-thread executor, 429 while busy: server.py:8, 39-40, 190-191). Here one worker process per
GPU owns its own pipeline, and the server hands each request to any idle worker. It answers 429
only when every worker is busy. Requests are independent, so nothing is exchanged between
GPUs (the frames / requests round-robin axis of multi-GPU serving).

Workers are started with the ``spawn`` method before the server process touches the GPU.
``start()`` refuses to run if this process has already initialised HIP: spawning re-executes
the interpreter, and exec from a GPU-initialised process is unsafe on this platform.
Images cross the process boundary as PNG bytes.
"""
from __future__ import annotations

import io
import multiprocessing as mp
import queue
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

from PIL import Image


def _to_png(img: Image.Image) -> bytes:
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return buf.getvalue()


def _from_png(b: bytes) -> Image.Image:
    return Image.open(io.BytesIO(b)).convert("RGB")


def _worker_main(rank: int, device_index: Optional[int], loader_spec: str, do_warmup: bool,
                 req_q, res_q):
    """Worker process: pin the GPU, load the pipeline, serve jobs until a None arrives."""
    try:
        import torch
        from .server import _import, process_image_sync, warmup
        if device_index is not None and torch.cuda.is_available():
            torch.cuda.set_device(device_index)
        pipe = _import(loader_spec)()
        if do_warmup:
            warmup(pipe)
        res_q.put(("ready", rank, None))
    except Exception as e:  # report and exit: the dispatcher marks this worker dead
        res_q.put(("dead", rank, f"{type(e).__name__}: {e}"))
        return
    while True:
        job = req_q.get()
        if job is None:
            break
        png, prompt, steps, use_cfg = job
        try:
            out = process_image_sync(pipe, _from_png(png), prompt, steps, use_cfg)
            res_q.put(("ok", rank, _to_png(out)))
        except Exception as e:
            res_q.put(("err", rank, f"{e}"))


class WorkerDied(RuntimeError):
    """The GPU worker serving a request exited (GPU fault, OOM kill) before it answered, or was
    terminated because the request passed its deadline (a hung worker)."""


class GpuDispatcher:
    """``size`` worker processes (one per GPU, device ``devices[i]``), one request each.

    Same worker protocol as ``server.LocalWorker``: ``try_acquire() -> token | None``,
    ``run(token, image, request)`` (blocking, on ``executor``), ``release(token)``.

    A worker that dies mid-request is detected while ``run`` waits (its process is polled every
    ``poll`` seconds): the request fails with ``WorkerDied`` (HTTP 500), the death is recorded in
    ``errors``, and a fresh ``spawn`` child is started for that GPU in the background (a new
    process, never an exec of this one). The slot stays out of the free list until the new worker
    reports ready, so a lost GPU never turns into a permanent 429.

    ``request_timeout`` (seconds, None = no deadline): a worker that is alive but has not answered
    by then (a stuck kernel, a deadlock) is terminated and takes the same path as a dead one --
    the request fails with ``WorkerDied`` and a fresh worker is spawned for the slot.
    """

    def __init__(self, size: int, loader_spec: str, devices: Optional[List[Optional[int]]] = None,
                 do_warmup: bool = True, start_timeout: float = 1800.0, poll: float = 1.0,
                 respawn: bool = True, request_timeout: Optional[float] = None):
        self.size = size
        self.loader_spec = loader_spec
        self.devices = list(devices) if devices is not None else list(range(size))
        self.do_warmup = do_warmup
        self.start_timeout = start_timeout
        self.poll = poll
        self.respawn = respawn
        self.request_timeout = request_timeout
        self.executor = ThreadPoolExecutor(max_workers=size)
        self._lock = threading.Lock()
        self._free: List[int] = []
        self._down = set()  # slots whose worker died; not handed out until a replacement is ready
        self._procs = []
        self._req = []
        self._res = []
        self._ctx = None
        self.errors = {}
        self.restarts = 0

    @property
    def loaded(self) -> bool:
        return bool(self._procs) and len(self.errors) < self.size

    def _spawn(self, r: int):
        rq, sq = self._ctx.Queue(), self._ctx.Queue()
        p = self._ctx.Process(target=_worker_main, args=(r, self.devices[r], self.loader_spec,
                                                         self.do_warmup, rq, sq), daemon=True)
        p.start()
        return p, rq, sq

    def _await_ready(self, r: int, sq) -> bool:
        try:
            kind, rank, msg = sq.get(timeout=self.start_timeout)
        except queue.Empty:
            kind, rank, msg = "dead", r, "timed out while loading"
        if kind == "ready":
            return True
        self.errors[r] = msg
        return False

    def start(self):
        import torch
        if torch.cuda.is_initialized():
            raise RuntimeError("GpuDispatcher.start() must run before this process touches the GPU")
        self._ctx = mp.get_context("spawn")
        for r in range(self.size):
            p, rq, sq = self._spawn(r)
            self._procs.append(p)
            self._req.append(rq)
            self._res.append(sq)
        for r in range(self.size):
            if self._await_ready(r, self._res[r]):
                self._free.append(r)

    def try_acquire(self) -> Optional[int]:
        with self._lock:
            return self._free.pop(0) if self._free else None

    def release(self, token: int):
        with self._lock:
            if token not in self._down:
                self._free.append(token)

    def _replace(self, token: int):
        """Start a fresh worker for ``token``'s GPU; the slot returns to the pool once it is ready."""
        import torch
        if torch.cuda.is_initialized():  # spawn re-executes the interpreter: never from a GPU process
            self.errors[token] = "worker died; not respawned (dispatcher process holds the GPU)"
            return
        p, rq, sq = self._spawn(token)
        self._procs[token], self._req[token], self._res[token] = p, rq, sq
        self.restarts += 1
        if self._await_ready(token, sq):
            with self._lock:
                self.errors.pop(token, None)
                self._down.discard(token)
                self._free.append(token)

    def _worker_died(self, token: int, why: Optional[str] = None):
        code = self._procs[token].exitcode
        with self._lock:
            self._down.add(token)
        self.errors[token] = why or f"worker {token} died (exit code {code})"
        try:
            self._procs[token].join(timeout=1)
        except Exception:
            pass
        if self.respawn:
            threading.Thread(target=self._replace, args=(token,), daemon=True).start()
        raise WorkerDied(self.errors[token])

    def run(self, token: int, image: Image.Image, req) -> Image.Image:
        self._req[token].put((_to_png(image), req.prompt, req.steps, req.use_cfg))
        res, proc = self._res[token], self._procs[token]
        deadline = None if self.request_timeout is None else time.monotonic() + self.request_timeout
        while True:
            try:
                kind, _, payload = res.get(timeout=self.poll)
                break
            except queue.Empty:
                if not proc.is_alive():
                    try:  # the answer may have landed just before the exit
                        kind, _, payload = res.get(timeout=0.1)
                        break
                    except queue.Empty:
                        self._worker_died(token)
                if deadline is not None and time.monotonic() > deadline:
                    # alive but silent past the deadline: end it (SIGTERM, then SIGKILL) and take
                    # the dead-worker path, which spawns a replacement
                    proc.terminate()
                    proc.join(timeout=5)
                    if proc.is_alive():
                        proc.kill()
                        proc.join(timeout=5)
                    self._worker_died(token, f"worker {token} died: no answer within {self.request_timeout:g} s "
                                             "(terminated)")
        if kind != "ok":
            raise RuntimeError(payload)
        return _from_png(payload)

    def stop(self):
        for q in self._req:
            q.put(None)
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self._procs, self._free = [], []
