"""Same-box yardstick for the exact path's score GEMM (a measurement only, never
on the product path): torch.matmul in fp16 (hipBLASLt) at configs[4]'s shape,
[1024 x 1536] queries x [1536 x 1M] rows -> 1024 x 1M fp32-accumulated scores
written as fp16 (2 GB of output writes, ~0.3 ms of HBM time inside the
kernel), random operands.
Run under rocprofv3 --kernel-trace --stats for the kernel's own duration.
Usage: python tools/gemm_yardstick.py [reps=20]"""
import sys
import time

import torch

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda")
B, d, n = 1024, 1536, 1_000_000
g = torch.Generator(device=dev)
g.manual_seed(1)
Q = (torch.rand(B, d, generator=g, device=dev) * 2 - 1).half()
X = (torch.rand(n, d, generator=g, device=dev) * 2 - 1).half()
flops = 2.0 * B * n * d
for name, fn in (("fp16_out", lambda: Q @ X.t()),):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{name}: {ms:.3f} ms/launch (HIP events) = {flops / ms / 1e9:.1f} TFLOP/s "
          f"= {flops / ms / 1e9 / 2500:.3f} of 2.5 PF", flush=True)
