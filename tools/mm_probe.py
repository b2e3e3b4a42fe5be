import torch
dev = "cuda"
for (M, K, N) in [(25600, 1792, 256), (25600, 1792, 128), (51200, 1792, 256), (25600, 256, 256), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(K, N, device=dev).to(torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 50
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    print(f"mm {M}x{K}x{N}: {us:.1f} us, {2*M*K*N/us/1e6:.0f} TF/s", flush=True)
