"""Calibration probe: hipBLASLt (torch.mm) bf16 GEMM rate at BASELINE config 5's two product
shapes (G1: [4096 x 1024] x [1024 x 16384], G2: [1024 x 4096] x [4096 x 16384]) and a plain
HBM copy rate; numbers only, nothing here is on the product path."""
import json
import torch

def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps

out = {}
B = 16384
for name, (M, K) in {"G1": (4096, 1024), "G2": (1024, 4096)}.items():
    W = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    S = torch.randn(K, B, device="cuda", dtype=torch.bfloat16)
    ms = t(lambda: torch.mm(W, S))
    out[name + "_bf16out_ms"] = ms
    out[name + "_bf16out_tflops"] = 2 * M * K * B / ms / 1e9
    C = torch.empty(M, B, device="cuda", dtype=torch.float32)
    ms = t(lambda: torch.mm(W, S, out_dtype=torch.float32) if hasattr(torch, "_scaled_mm") and False else torch.mm(W.float(), S.float(), out=C))
    out[name + "_f32_ms"] = ms
x = torch.empty(256 << 20, device="cuda", dtype=torch.float32)
y = torch.empty_like(x)
ms = t(lambda: y.copy_(x))
out["copy_GBps"] = 2 * x.numel() * 4 / ms / 1e6
print(json.dumps(out))
