import torch, time
dev = torch.device("cuda:0")
for name, (M, N, K) in {"up": (16384, 12288, 3072), "qkv": (16384, 9216, 3072), "down": (16384, 3072, 12288)}.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
    for _ in range(5):
        c = a @ b.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(10):
        e0.record()
        for _ in range(5):
            c = a @ b.t()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    ts.sort()
    print(f"torch.matmul {name}: median {ts[5]:.3f} ms  {2*M*N*K/ts[5]/1e9:.0f} TFLOP/s")
