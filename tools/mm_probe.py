import torch, time, sys
sys.path.insert(0, '.')
from qwen_image_edit_streamdiffusion_amd import ops
dev='cuda'
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)/it
for name,M,N,K in [("qkv",16384,9216,3072),("out",16384,3072,3072),("up",16384,12288,3072),("down",16384,3072,12288)]:
    x=torch.randn(M,K,device=dev).to(torch.bfloat16); w=torch.randn(N,K,device=dev).to(torch.bfloat16)/60
    b=torch.zeros(N,device=dev,dtype=torch.bfloat16)
    out=torch.empty(M,N,device=dev,dtype=torch.bfloat16)
    t_lib=bench(lambda: torch.mm(x, w.t(), out=out))
    t_f=bench(lambda: torch.nn.functional.linear(x, w, b))
    t_me=bench(lambda: ops.linear(x,w,b,out=out))
    fl=2*M*N*K
    print(f"{name}: torch.mm {t_lib*1e3:.0f}us {fl/t_lib/1e9:.0f}TF  F.linear {t_f*1e3:.0f}us {fl/t_f/1e9:.0f}TF  qie {t_me*1e3:.0f}us {fl/t_me/1e9:.0f}TF")
