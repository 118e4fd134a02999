"""Does ROCr's HSA_CU_MASK restrict this process's queues? Times a bf16 GEMM (compute-bound: the
time scales with the compute units a process may use)."""
import sys
import time

import torch

a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    a @ b
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    a @ b
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 10
print(sys.argv[1] if len(sys.argv) > 1 else "", f"{dt * 1e3:.2f} ms", f"{2 * 8192 ** 3 / dt / 1e12:.0f} TF/s", flush=True)
