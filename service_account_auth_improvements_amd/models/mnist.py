"""MNIST CNN for BASELINE configs[0] ("PyTorchJob 2-worker MNIST on CPU/gloo via local kind
cluster") -- the control-plane plumbing job (the reference conformance suite runs the
training-operator's MNIST image).  Synthetic MNIST-shaped data (no downloads): 28x28
images whose class is encoded in a fixed per-class pattern plus noise, so the loss falls.

Training is plain torch DDP (gloo on CPU, RCCL on GPU) -- this job exists to exercise the
operator, launcher and rendezvous, not the MI355X kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class MnistNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.c1 = nn.Conv2d(1, 16, 5, padding=2)
        self.c2 = nn.Conv2d(16, 32, 5, padding=2)
        self.fc = nn.Linear(32 * 7 * 7, 10)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.c1(x)), 2)
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        return self.fc(x.flatten(1))


class SyntheticMnist:
    def __init__(self, batch: int, device, seed: int = 0, rank: int = 0):
        g = torch.Generator().manual_seed(1234)
        self.protos = torch.randn(10, 1, 28, 28, generator=g)
        self.g = torch.Generator().manual_seed(seed * 1000 + rank)
        self.batch, self.device = batch, device

    def next(self):
        y = torch.randint(0, 10, (self.batch,), generator=self.g)
        x = self.protos[y] + 0.5 * torch.randn(self.batch, 1, 28, 28, generator=self.g)
        return x.to(self.device), y.to(self.device)


class MnistTrainer:
    def __init__(self, device, lr: float = 0.05):
        import torch.distributed as dist
        torch.manual_seed(0)
        self.model = MnistNet().to(device)
        if dist.is_initialized() and dist.get_world_size() > 1:
            self.model = nn.parallel.DistributedDataParallel(self.model)
        self.opt = torch.optim.SGD(self.model.parameters(), lr=lr, momentum=0.9)
        self.step_idx = 0

    def _module(self):
        return self.model.module if hasattr(self.model, "module") else self.model

    def state_tensors(self) -> dict:
        """Weights and SGD momentum buffers as a flat name -> tensor dict (safetensors)."""
        out = {f"w/{k}": v.detach() for k, v in self._module().state_dict().items()}
        for i, p in enumerate(self._module().parameters()):
            buf = self.opt.state.get(p, {}).get("momentum_buffer")
            if buf is not None:
                out[f"momentum/{i}"] = buf.detach()
        return out

    def load_state_tensors(self, t: dict):
        m = self._module()
        m.load_state_dict({k[2:]: v for k, v in t.items() if k.startswith("w/")})
        for i, p in enumerate(m.parameters()):
            if f"momentum/{i}" in t:
                self.opt.state[p]["momentum_buffer"] = t[f"momentum/{i}"].to(p.device).clone()

    def train_step(self, batches):
        """One optimizer step over a list of micro-batches (gradient accumulation)."""
        self.opt.zero_grad(set_to_none=True)
        tot = None
        for x, y in batches:
            loss = F.cross_entropy(self.model(x), y) / len(batches)
            loss.backward()
            tot = loss.detach() if tot is None else tot + loss.detach()
        self.opt.step()
        self.step_idx += 1
        return tot
