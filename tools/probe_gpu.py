"""One-off hardware probe: device props, GEMM TFLOP/s on Llama-3-8B shapes, SDPA speed."""
import time, torch, json, os
import torch.nn.functional as F
d = torch.device("cuda:0")
p = torch.cuda.get_device_properties(0)
print("device", p.name, p.gcnArchName, p.total_memory/2**30, "GiB", p.multi_processor_count, "CUs")
def bench(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-t)/it
T=8192
for (M,N,K) in [(T,6144,4096),(T,4096,4096),(T,28672,4096),(T,4096,14336),(T,128256,4096),(4096,14336,T)]:
    a=torch.randn(M,K,device=d,dtype=torch.bfloat16); b=torch.randn(N,K,device=d,dtype=torch.bfloat16)
    t=bench(lambda: a@b.t()); print(f"gemm {M}x{N}x{K}: {t*1e3:.3f} ms {2*M*N*K/t/1e12:.0f} TF")
for S in [4096, 8192]:
    q=torch.randn(1,32,S,128,device=d,dtype=torch.bfloat16,requires_grad=True)
    k=torch.randn(1,8,S,128,device=d,dtype=torch.bfloat16,requires_grad=True)
    v=torch.randn(1,8,S,128,device=d,dtype=torch.bfloat16,requires_grad=True)
    f=lambda: F.scaled_dot_product_attention(q,k,v,is_causal=True,enable_gqa=True)
    t=bench(f); fl=4*S*S*128*32/2
    print(f"sdpa fwd S={S}: {t*1e3:.3f} ms {fl/t/1e12:.0f} TF")
    o=f(); g=torch.randn_like(o)
    def fb():
        o=f(); o.backward(g)
    t2=bench(fb); print(f"sdpa fwd+bwd S={S}: {t2*1e3:.3f} ms {3.5*fl/t2/1e12:.0f} TF")
x=torch.randn(2**28,device=d)
t=bench(lambda: x.mul_(1.0001)); print(f"copy-ish BW {2*x.numel()*4/t/1e12:.2f} TB/s")
print(torch.backends.cuda.flash_sdp_enabled(), torch.backends.cuda.mem_efficient_sdp_enabled())
