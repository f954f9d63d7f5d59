"""First-use costs inside a fresh trainer process (what CRD-to-first-step's init_to_first_step
holds beyond the step itself): torch import, device init, first hipBLASLt GEMM, first HIP-kernel
launch, and the first vs second training step of the Llama-3-8B trainer at micro-batch 1."""
import json
import os
import sys
import time

t0 = time.perf_counter()
import torch  # noqa: E402
t_import = time.perf_counter() - t0
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = {"import_torch_s": round(t_import, 3)}
t = time.perf_counter()
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
out["device_init_s"] = round(time.perf_counter() - t, 3)
a = torch.randn(256, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
for name in ("first_gemm_s", "second_gemm_same_shape_s"):
    t = time.perf_counter()
    torch.mm(a, w.t())
    torch.cuda.synchronize()
    out[name] = round(time.perf_counter() - t, 4)
t = time.perf_counter()
torch.mm(torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16), w.t())
torch.cuda.synchronize()
out["new_shape_gemm_s"] = round(time.perf_counter() - t, 4)
t = time.perf_counter()
from service_account_auth_improvements_amd.ops import _ext  # noqa: E402
from service_account_auth_improvements_amd import ops  # noqa: E402
_ext.load()
x = torch.randn(64, 4096, device="cuda", dtype=torch.bfloat16)
ops.rmsnorm_fwd(x, torch.ones(4096, device="cuda", dtype=torch.bfloat16), 1e-5)
torch.cuda.synchronize()
out["ext_load_first_kernel_s"] = round(time.perf_counter() - t, 4)
from service_account_auth_improvements_amd.parallel.state import ParallelState  # noqa: E402
from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer  # noqa: E402
t = time.perf_counter()
tr = Trainer(TrainConfig(model="llama3-8b", seq_len=8192, micro_batch=1), ParallelState(device=torch.device("cuda", 0)))
torch.cuda.synchronize()
out["trainer_init_s"] = round(time.perf_counter() - t, 3)
data = SyntheticData(tr.mcfg.vocab_size, 1, 8192, torch.device("cuda", 0), seed=1)
for k in range(3):
    b = [data.next()]
    t = time.perf_counter()
    tr.train_step(b)
    torch.cuda.synchronize()
    out[f"step{k + 1}_s"] = round(time.perf_counter() - t, 3)
print(json.dumps(out))
