"""Stub pipelines for the /edit server tests (CPU only; imported by spawned dispatcher workers
through the loader spec "server_stubs:load_stub", so it must stay importable by module name)."""
import time

from PIL import Image, ImageOps


class _Out:
    def __init__(self, images):
        self.images = images


class StubPipeline:
    """Records every call; returns the inverted input image after ``delay`` seconds."""

    def __init__(self, delay: float = 0.0, fail: str = "", die_on: str = "", hang_on: str = ""):
        self.calls = []
        self.delay = delay
        self.fail = fail
        self.die_on = die_on
        self.hang_on = hang_on

    def __call__(self, **kw):
        self.calls.append(kw)
        if self.die_on and kw.get("prompt") == self.die_on:
            import os
            os._exit(3)  # a worker lost mid-request (GPU fault / OOM kill stand-in)
        if self.hang_on and kw.get("prompt") == self.hang_on:
            while True:  # a worker that stays alive and never answers (stuck kernel stand-in)
                time.sleep(3600)
        if self.fail:
            raise ValueError(self.fail)
        if self.delay:
            time.sleep(self.delay)
        return _Out([ImageOps.invert(kw["image"][0])])


def load_stub():
    return StubPipeline(delay=1.5)


def load_dying_stub():
    return StubPipeline(delay=0.2, die_on="die")


def load_hanging_stub():
    return StubPipeline(delay=0.1, hang_on="hang")


def solid(color, size=(64, 48)):
    return Image.new("RGB", size, color=color)
