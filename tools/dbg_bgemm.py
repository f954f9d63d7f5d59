import torch, sys
sys.path.insert(0, "/root/repo")
from service_account_auth_improvements_amd import ops
torch.manual_seed(0)
for K in (2048, 4096):
  for M in (17, 65, 128, 129, 200):
    for sw in (False, True):
        Nw = 512
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(Nw, K, device="cuda") * 0.05).bfloat16()
        ref = torch.mm(x.float(), w.float().t())
        if sw: ref = torch.nn.functional.silu(ref[:, :Nw // 2]) * ref[:, Nw // 2:]
        line = f"K={K} M={M} sw={int(sw)}:"
        for S in (1, 2, 4, 8):
            if (K // 256) % S: continue
            y = ops.bgemm(x, w, swiglu=sw, splits=S).float()
            e = ((y - ref).abs().max() / ref.abs().max()).item()
            line += f" S{S}={e:.1e}"
            if e > 1e-2:
                bad = ((y - ref).abs() > 0.05 * ref.abs().max())
                rows = bad.any(1).nonzero().flatten().tolist(); cols = bad.any(0).nonzero().flatten().tolist()
                line += f"[rows {rows[:4]}..{len(rows)} cols {cols[:6]}..{len(cols)}]"
        print(line, flush=True)
