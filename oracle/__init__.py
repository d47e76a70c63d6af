"""CPU oracle for the Qwen-Image-Edit-2509 denoise hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package, and only as the
checker / the timed CPU baseline.  The product path
(``qwen_image_edit_streamdiffusion_amd``) never imports it and fails loudly
when its HIP library is missing.

PARITY UNPINNED: the reference (shi3z/Qwen-Image-Edit-StreamDiffusion) holds no
golden vectors, no asserts and no source for the hot-path arithmetic; that lives
in the un-vendored third-party package ``diffusers`` (unpinned, README.md:49),
which is absent from this container, as are the model weights.  The modules here
restate the published upstream algorithm and are pinned
only by closed-form known answers (sigma schedule, RoPE, timestep embedding) and
by invariants.
"""
