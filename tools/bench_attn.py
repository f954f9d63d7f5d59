"""Attention microbench: HIP flash kernels vs torch SDPA at Llama-3-8B shapes."""
import math, sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from service_account_auth_improvements_amd.ops import _ext
from service_account_auth_improvements_amd.ops.attention import _split
_ext.load()
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/it
B,Hq,Hkv,D=1,32,8,128
for S in [int(x) for x in (sys.argv[1:] or ["4096","8192"])]:
    qkv=torch.randn(B*S,(Hq+2*Hkv)*D,device="cuda",dtype=torch.bfloat16)
    fl=4*S*S*D*Hq/2*B
    t=bench(lambda: torch.ops.kfamd.flash_fwd(qkv,B,S,Hq,Hkv,D,1/math.sqrt(D),True))
    print(f"S={S} hip fwd {t*1e3:.3f} ms {fl/t/1e12:.0f} TF")
    q,k,v=(x.contiguous() for x in _split(qkv,B,S,Hq,Hkv,D))
    t=bench(lambda: F.scaled_dot_product_attention(q,k,v,is_causal=True,enable_gqa=True))
    print(f"S={S} sdpa fwd {t*1e3:.3f} ms {fl/t/1e12:.0f} TF")
    if hasattr(torch.ops.kfamd, "flash_bwd"):
        o,lse=torch.ops.kfamd.flash_fwd(qkv,B,S,Hq,Hkv,D,1/math.sqrt(D),True)
        do=torch.randn_like(o)
        t=bench(lambda: torch.ops.kfamd.flash_bwd(qkv,o,lse,do,B,S,Hq,Hkv,D,1/math.sqrt(D),True))
        print(f"S={S} hip bwd {t*1e3:.3f} ms {2.5*fl/t/1e12:.0f} TF")
