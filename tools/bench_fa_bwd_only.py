"""Run only the flash bwd at S=8192 a few times (for PMC collection)."""
import math, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from service_account_auth_improvements_amd.ops import _ext
_ext.load()
B,Hq,Hkv,D,S=1,32,8,128,int(sys.argv[1]) if len(sys.argv)>1 else 8192
qkv=torch.randn(B*S,(Hq+2*Hkv)*D,device="cuda",dtype=torch.bfloat16)
o,lse=torch.ops.kfamd.flash_fwd(qkv,B,S,Hq,Hkv,D,1/math.sqrt(D),True)
do=torch.randn_like(o)
for _ in range(3):
    torch.ops.kfamd.flash_bwd(qkv,o,lse,do,B,S,Hq,Hkv,D,1/math.sqrt(D),True,False)
torch.cuda.synchronize()
