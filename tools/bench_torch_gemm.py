"""Ceiling check: hipBLASLt (torch.matmul, bf16) on the 1x1-conv GEMM shapes of
res2net50_w24_s4_c32 at B=256, 80x200 -- a library reference point for
gemm1x1_pipe (no BN/residual epilogue, so it moves fewer bytes)."""
import json
import torch

B = 256
shapes = {
    "L2_1x1c": (B * 4000, 192, 256), "L2_1x1a": (B * 4000, 256, 192),
    "L3_1x1a": (B * 1000, 512, 384), "L3_1x1c": (B * 1000, 384, 512),
    "L4_1x1a": (B * 250, 1024, 768), "L4_1x1c": (B * 250, 768, 1024),
    "L3_proj": (B * 1000, 256, 512), "L4_proj": (B * 250, 512, 1024),
}
dev = torch.device("cuda", 0)
out = {}
for name, (M, K, N) in shapes.items():
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        torch.matmul(a, w, out=c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        torch.matmul(a, w, out=c)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    fl = 2.0 * M * K * N
    by = 2.0 * (M * K + K * N + M * N)
    out[name] = {"M": M, "K": K, "N": N, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1),
                 "gbs": round(by / us / 1e3, 1)}
    print(name, out[name], flush=True)
# plain copy bandwidth
x = torch.empty(512 * 1024 * 1024, dtype=torch.uint8, device=dev)
y = torch.empty_like(x)
for _ in range(3):
    y.copy_(x)
torch.cuda.synchronize()
e0.record()
for _ in range(10):
    y.copy_(x)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 10 * 1e3
out["copy_512MiB"] = {"us": round(us, 1), "gbs": round(2 * x.numel() / us / 1e3, 1)}
print(json.dumps(out))
