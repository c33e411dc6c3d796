"""What do the vendor f32 GEMMs (torch.mm -> hipBLASLt/rocBLAS) reach on the same shapes? (diagnostic ceiling)"""
import torch

PEAK = 157.3


def t(fn, it=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it


torch.backends.cuda.matmul.allow_tf32 = False
for M, N, K in [(4096, 256, 768), (8192, 256, 768), (4096, 256, 256), (4096, 256, 2048), (256, 768, 4096),
                (256, 768, 8192), (4096, 4096, 4096), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    us = t(lambda: torch.mm(a, b))
    tf = 2 * M * N * K / us / 1e6
    print(f"torch.mm f32 {M}x{N}x{K}: {us:8.2f} us {tf:7.2f} TF/s {tf / PEAK:.3f}", flush=True)
