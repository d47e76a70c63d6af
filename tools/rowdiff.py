"""Where does a batch row stop being independent of its batch? Runs a 1-block full-width model on
a B = 2 input and on row r alone, and compares every workspace buffer of the two runs on that
row's slice (first differing stage = the kernel to look at). Debug tool, GPU only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from qwen_image_edit_streamdiffusion_amd import QwenImageTransformer2DModel  # noqa: E402

BF16 = torch.bfloat16
S_IMG, S_TXT = 8192, 216
SHAPES = [(1, 64, 64), (1, 64, 64)]


def snap(m, key):
    ws = m._ws[key]
    names = ["x_img", "x_txt", "h_img", "h_txt", "att_img", "att_txt", "mlp_img", "mlp_txt", "qkv", "mod_all",
             "emb_out", "temb", "stemb", "txt_norm"]
    return {n: getattr(ws, n).clone() for n in names}


def main():
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dev = torch.device("cuda")
    m = QwenImageTransformer2DModel(num_layers=layers, device=dev).random_init_(seed=0)
    if len(sys.argv) > 2 and sys.argv[2] == "int8":
        m.quantize_int8()
    g = torch.Generator(device=dev).manual_seed(11)
    hs = torch.randn(2, S_IMG, 64, generator=g, device=dev).to(BF16)
    enc = torch.randn(2, S_TXT, 3584, generator=g, device=dev).to(BF16)
    lens = [S_TXT, S_TXT]
    t = (torch.tensor([1000.0, 20.0]).to(BF16) / 1000).to(BF16).to(dev)
    a = m(hs, enc, None, t, [SHAPES] * 2, lens, return_dict=False)[0].clone()
    sa = snap(m, (2, S_IMG, S_TXT, m.int8))
    for r in (0, 1):
        o = m(hs[r:r + 1], enc[r:r + 1], None, t[r:r + 1], [SHAPES], lens[r:r + 1], return_dict=False)[0].clone()
        sb = snap(m, (1, S_IMG, S_TXT, m.int8))
        print(f"row {r}: out equal {torch.equal(o, a[r:r + 1])}")
        for n, vb in sb.items():
            va = sa[n]
            if n == "qkv":
                va = va[:, r:r + 1]
            else:
                rows = vb.shape[0]
                va = va[r * rows:(r + 1) * rows]
            eq = torch.equal(va, vb)
            d = (va.float() - vb.float())
            nz = (d != 0)
            print(f"   {n:8s} equal={eq}  ndiff={int(nz.sum())}  maxabs={d.abs().max().item():.3e}"
                  + (f"  first_diff_index={nz.nonzero()[0].tolist()}" if not eq else ""))


if __name__ == "__main__":
    main()
