import torch, time
dev = torch.device("cuda:0")
for (N, H, V) in ((6144, 768, 50257), (16384, 4096, 32128), (24576, 768, 32128)):
    h = torch.randn(N, H, device=dev, dtype=torch.bfloat16)
    W = torch.randn(V, H, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        y = h @ W.t()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        y = h @ W.t()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"N={N} H={H} V={V}: {ms*1e3:.1f} us  {2*N*H*V/ms/1e9:.1f} TFLOP/s  out {y.numel()*2/1e6:.0f} MB")
