"""Time the prompt encoder at Qwen2.5-VL-7B size on random bf16 weights: the
vision tower on one 392x392 condition image (28x28 patches -> 196 image tokens) and the language
model on the Edit-Plus prompt around it (S tokens). Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from qwen_image_edit_streamdiffusion_amd.text_encoder import (QwenVLEncoder, TextEncoderConfig,  # noqa: E402
                                                              random_state_dict, text_state_dict_shapes)
from qwen_image_edit_streamdiffusion_amd.vision import VisionConfig, vision_state_dict_shapes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=300)
    ap.add_argument("--grid", type=int, default=28)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    tc, vc = TextEncoderConfig(), VisionConfig()
    sd = {"model.language_model." + k: v for k, v in random_state_dict(text_state_dict_shapes(tc), dev, 0).items()}
    sd.update({"model.visual." + k: v for k, v in random_state_dict(vision_state_dict_shapes(vc), dev, 1).items()})
    enc = QwenVLEncoder(tc, vc, dev).load_state_dict(sd)
    del sd
    torch.cuda.empty_cache()
    n_img = (a.grid // 2) ** 2
    S = a.tokens
    ids = torch.randint(0, 150000, (S,))
    ids[70:70 + n_img] = enc.image_token_id
    grid = [(1, a.grid, a.grid)]
    pv = torch.randn(a.grid * a.grid, vc.patch_dim)
    res = {}
    for name, fn in (("vision", lambda: enc.vision(pv, grid)),
                     ("text", lambda: enc.text(ids)),
                     ("encoder", lambda: enc(ids, pv, grid))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        res[name + "_ms"] = round((time.perf_counter() - t0) / a.iters * 1e3, 2)
    Sp = -(-S // 64) * 64
    D, F, L = tc.hidden_size, tc.intermediate_size, tc.num_hidden_layers
    kv = tc.num_key_value_heads * tc.head_dim
    text_flops = L * (2 * Sp * D * (D + 2 * kv + D + 3 * F) + tc.num_attention_heads * 4 * Sp * Sp * tc.head_dim)
    vis_flops = enc.vision.flops(a.grid * a.grid)
    res.update(text_tflops=round(text_flops / res["text_ms"] / 1e9, 1),
               vision_tflops=round(vis_flops / res["vision_ms"] / 1e9, 1),
               tokens=S, image_tokens=n_img, config="Qwen2.5-VL-7B (random bf16 weights)")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
