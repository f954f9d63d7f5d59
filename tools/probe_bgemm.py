"""A few batched-decode GEMM calls of one shape for counter collection (tools/gpu_session.sh
pmctool): ops.bgemm and hipBLASLt (torch.mm) on fresh weight copies.

    python tools/probe_bgemm.py [M N K reps]      (default: 128 4096 14336 10 -- the wd projection)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from service_account_auth_improvements_amd import ops  # noqa: E402


def main():
    M, N, K, reps = (int(a) for a in (sys.argv[1:5] if len(sys.argv) >= 5 else (128, 4096, 14336, 10)))
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(max(2, (1 << 30) // (N * K * 2)))]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for i in range(reps):
        ops.bgemm(x, ws[i % len(ws)])
        torch.mm(x, ws[(i + 1) % len(ws)].t())
    torch.cuda.synchronize()
    print(f"bgemm / hipBLASLt x {reps}: M {M} N {N} K {K}")


if __name__ == "__main__":
    main()
