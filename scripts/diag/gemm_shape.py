"""Diagnostic: torch (hipBLASLt) fp32 GEMM time for config 4's A_1 = X Omega_1 shape
([B x 784] @ [784 x 4096]) next to the engine's k_step_agemm, HIP events over 200 launches."""
import torch

dev = torch.device("cuda", 0)
for M in (200, 224, 10000):
    X = torch.randn(M, 784, device=dev)
    Om = torch.randn(784, 4096, device=dev)
    out = torch.empty(M, 4096, device=dev)
    for _ in range(20):
        torch.mm(X, Om, out=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record()
    for _ in range(n):
        torch.mm(X, Om, out=out)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    fl = 2 * M * 784 * 4096
    print(f"M={M}: {us:.1f} us/GEMM, {fl / us / 1e6:.1f} TFLOP/s", flush=True)
