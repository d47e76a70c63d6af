"""/edit serving surface against the reference's server.py contract, on the
CPU with a stub pipeline: routes, codec (data-URL prefix, EXIF transpose, JPEG q90), request
defaults (512x512 LANCZOS, seed 42, negative_prompt "" iff use_cfg), ref-image blend, and the
503 / 429 / 500 behaviour; plus the two-worker process dispatcher (spawned CPU workers). The
HIP pipeline behind the same app is exercised in test_gpu_server.py."""
import base64
import io
import threading

import numpy as np
import pytest
from PIL import Image

from qwen_image_edit_streamdiffusion_amd import server as S
from server_stubs import StubPipeline, solid

fastapi = pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402


def b64_png(img):
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    return base64.b64encode(buf.getvalue()).decode()


def decode_b64(s):
    return Image.open(io.BytesIO(base64.b64decode(s)))


def client_for(pipe):
    return TestClient(S.create_app(loader=lambda: pipe, do_warmup=False))


def test_root_and_health():
    with client_for(StubPipeline()) as c:
        r = c.get("/").json()
        assert r["endpoints"] == ["/health", "/edit"] and r["status"] == "running"
        h = c.get("/health").json()
        assert h["status"] == "ok" and h["model_loaded"] is True


def test_edit_cond_only_defaults():
    pipe = StubPipeline()
    with client_for(pipe) as c:
        r = c.post("/edit", json={"image": b64_png(solid((10, 200, 30)))})
        assert r.status_code == 200, r.text
        body = r.json()
        assert body["status"] == "success" and body["elapsed"] >= 0
        out = decode_b64(body["image"])
        assert out.format == "JPEG" and out.size == (512, 512)
        px = np.asarray(out.convert("RGB")).astype(int).mean(axis=(0, 1))
        assert np.allclose(px, [245, 55, 225], atol=3)  # the stub inverts
    kw = pipe.calls[0]
    assert kw["prompt"] == "Transform into oil painting style" and kw["num_inference_steps"] == 2
    assert kw["image"][0].size == (512, 512) and "negative_prompt" not in kw
    assert kw["guidance_scale"] == 3.5
    assert kw["generator"].initial_seed() == 42


def test_edit_cfg_steps_and_data_url():
    pipe = StubPipeline()
    with client_for(pipe) as c:
        r = c.post("/edit", json={"image": "data:image/png;base64," + b64_png(solid("white")),
                                  "prompt": "make it night", "steps": 4, "use_cfg": True})
        assert r.status_code == 200, r.text
    kw = pipe.calls[0]
    assert kw["negative_prompt"] == "" and kw["num_inference_steps"] == 4 and kw["prompt"] == "make it night"


def test_ref_image_blend():
    a, b = solid((200, 0, 0), (300, 200)), solid((0, 0, 200), (100, 100))
    req = S.EditRequest(image=b64_png(a), ref_image=b64_png(b), blend_ratio=0.25)
    out = S.prepare_input(S.Codec(), req)
    assert out.size == (512, 512)
    assert np.allclose(np.asarray(out).reshape(-1, 3).mean(0), [150, 0, 50], atol=1)


def test_exif_transpose():
    img = Image.new("RGB", (40, 20), "red")
    exif = Image.Exif()
    exif[0x0112] = 6  # rotate 90 degrees on display
    buf = io.BytesIO()
    img.save(buf, format="JPEG", exif=exif)
    out = S.base64_to_pil(base64.b64encode(buf.getvalue()).decode())
    assert out.size == (20, 40) and out.mode == "RGB"


def test_503_when_not_loaded():
    def bad_loader():
        raise RuntimeError("no weights")
    with TestClient(S.create_app(loader=bad_loader, do_warmup=False)) as c:
        r = c.post("/edit", json={"image": b64_png(solid("gray"))})
        assert r.status_code == 503 and r.json()["detail"] == "Model not loaded"
        assert "no weights" in c.get("/health").json()["load_error"]


def test_500_carries_the_error():
    with client_for(StubPipeline(fail="boom")) as c:
        r = c.post("/edit", json={"image": b64_png(solid("gray"))})
        assert r.status_code == 500 and r.json()["detail"] == "boom"
        # a bad base64 payload is a 500 as well (the reference decodes inside its try)
        r = c.post("/edit", json={"image": "not-an-image"})
        assert r.status_code == 500


def test_429_while_busy():
    gate = threading.Event()

    class Blocking(StubPipeline):
        def __call__(self, **kw):
            gate.wait(10)
            return super().__call__(**kw)

    with client_for(Blocking()) as c:
        first = {}
        t = threading.Thread(target=lambda: first.update(r=c.post("/edit", json={"image": b64_png(solid("gray"))})))
        t.start()
        import time
        for _ in range(200):  # wait until the first request holds the worker
            if c.app.state.qie["worker"].try_acquire() is None:
                break
            c.app.state.qie["worker"].release(0)
            time.sleep(0.01)
        r = c.post("/edit", json={"image": b64_png(solid("gray"))})
        assert r.status_code == 429
        gate.set()
        t.join(10)
        assert first["r"].status_code == 200


def test_gpu_dispatcher_two_workers_cpu():
    """Two spawned workers (CPU stubs, 1.5 s per request): two concurrent requests are served
    in parallel, a third one meanwhile gets 429."""
    from qwen_image_edit_streamdiffusion_amd.dispatch import GpuDispatcher
    d = GpuDispatcher(2, "server_stubs:load_stub", devices=[None, None], do_warmup=False,
                      start_timeout=300)
    with TestClient(S.create_app(dispatcher=d)) as c:
        assert c.get("/health").json()["workers"] == 2
        res = {}

        def go(i):
            res[i] = c.post("/edit", json={"image": b64_png(solid("gray")), "prompt": f"p{i}"})
        ts = [threading.Thread(target=go, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        import time
        time.sleep(0.5)
        r3 = c.post("/edit", json={"image": b64_png(solid("gray"))})
        for t in ts:
            t.join(60)
        assert r3.status_code == 429
        assert res[0].status_code == 200 and res[1].status_code == 200
        assert decode_b64(res[0].json()["image"]).size == (512, 512)


def test_gpu_dispatcher_worker_death_is_500_and_respawned():
    """A worker that dies mid-request fails that request with 500 (not a hang),
    is recorded in the health errors, and a fresh worker takes its slot (no permanent 429)."""
    import time
    from qwen_image_edit_streamdiffusion_amd.dispatch import GpuDispatcher
    d = GpuDispatcher(1, "server_stubs:load_dying_stub", devices=[None], do_warmup=False,
                      start_timeout=300, poll=0.2)
    with TestClient(S.create_app(dispatcher=d)) as c:
        r = c.post("/edit", json={"image": b64_png(solid("gray")), "prompt": "die"})
        assert r.status_code == 500 and "died" in r.json()["detail"]
        for _ in range(600):  # the replacement loads in the background
            if d.restarts == 1 and not d.errors and d.try_acquire() is not None:
                d.release(0)
                break
            time.sleep(0.1)
        assert d.restarts == 1 and not d.errors
        r = c.post("/edit", json={"image": b64_png(solid("gray")), "prompt": "ok"})
        assert r.status_code == 200


def test_gpu_dispatcher_hung_worker_hits_deadline_and_is_respawned():
    """A worker that stays alive but never answers: the request fails with 500 once its deadline
    passes, the worker is terminated, and a fresh one takes the slot (no permanent 429)."""
    import time
    from qwen_image_edit_streamdiffusion_amd.dispatch import GpuDispatcher
    d = GpuDispatcher(1, "server_stubs:load_hanging_stub", devices=[None], do_warmup=False,
                      start_timeout=300, poll=0.2, request_timeout=1.5)
    with TestClient(S.create_app(dispatcher=d)) as c:
        t0 = time.time()
        r = c.post("/edit", json={"image": b64_png(solid("gray")), "prompt": "hang"})
        assert r.status_code == 500 and "no answer within" in r.json()["detail"]
        assert time.time() - t0 < 30
        for _ in range(600):
            if d.restarts == 1 and not d.errors and d.try_acquire() is not None:
                d.release(0)
                break
            time.sleep(0.1)
        assert d.restarts == 1 and not d.errors
        r = c.post("/edit", json={"image": b64_png(solid("gray")), "prompt": "ok"})
        assert r.status_code == 200
