"""Library GEMM reference point (torch.matmul -> hipBLASLt, bf16) for the conv
GEMM shapes: what a plain GEMM of the same M x N x K reaches on this box."""
import torch
shapes = [('l4.c2', 32768, 512, 4608), ('l3.c2', 131072, 256, 2304), ('l2.c2', 524288, 128, 1152),
          ('l1.c', 2097152, 64, 576), ('big', 16384, 16384, 16384)]
for name, M, N, K in shapes:
    a = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(K, N, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); c = a @ b; e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts)[5] * 1e-3
    print(f'{name:6s} M={M} N={N} K={K}: {t*1e6:8.1f} us {2*M*N*K/t/1e12:7.1f} TF/s', flush=True)
