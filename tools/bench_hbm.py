"""HBM calibration on the box: read-only, write-only and copy rates of torch's
own kernels on 2 GiB buffers (context for the roofline fractions)."""
import json
import torch

dev = torch.device("cuda", 0)
n = 1 << 30
x = torch.ones(n, dtype=torch.bfloat16, device=dev)
y = torch.empty_like(x)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def t(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


out = {}
out["read_sum_GBs"] = 2 * n / t(lambda: x.sum(dtype=torch.float32)) / 1e9
out["write_fill_GBs"] = 2 * n / t(lambda: y.fill_(3.0)) / 1e9
out["copy_GBs"] = 4 * n / t(lambda: y.copy_(x)) / 1e9
out["add_GBs"] = 6 * n / t(lambda: torch.add(x, x, out=y)) / 1e9
print(json.dumps({k: round(v, 1) for k, v in out.items()}))
