"""Calibration: torch.matmul (hipBLASLt) f16 / bf16 throughput at the c5 GEMM shapes, for comparison
with the split-fp16 kernels (3 f16 MFMA products per fp32-accurate FLOP)."""
import torch

d = torch.device("cuda", 0)
for dt in (torch.float16, torch.bfloat16):
    for (M, N, K) in ((65536, 2048, 2048), (2048, 2048, 65536)):
        a = torch.randn(M, K, device=d, dtype=dt)
        b = torch.randn(K, N, device=d, dtype=dt)
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            c = a @ b
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{dt} {M}x{N}x{K}: {ms:.3f} ms  {2 * M * N * K / ms / 1e9:.0f} TFLOP/s", flush=True)
