"""Stub pipelines for the /edit server tests (CPU only; imported by spawned dispatcher workers
through the loader spec "server_stubs:load_stub", so it must stay importable by module name)."""
import time

from PIL import Image, ImageOps


class _Out:
    def __init__(self, images):
        self.images = images


class StubPipeline:
    """Records every call; returns the inverted input image after ``delay`` seconds."""

    def __init__(self, delay: float = 0.0, fail: str = ""):
        self.calls = []
        self.delay = delay
        self.fail = fail

    def __call__(self, **kw):
        self.calls.append(kw)
        if self.fail:
            raise ValueError(self.fail)
        if self.delay:
            time.sleep(self.delay)
        return _Out([ImageOps.invert(kw["image"][0])])


def load_stub():
    return StubPipeline(delay=1.5)


def solid(color, size=(64, 48)):
    return Image.new("RGB", size, color=color)
