"""Tensor-parallel predictor: one InferenceService pod over ``amd.com/gpu: N`` GPUs.

The predictor pod runs ``kfamd-launch --nproc-per-node N --isolate-devices -- python -m
...serving.server --tp N`` (controlplane/inferenceservice.py), i.e. one process per GPU,
each holding a 1/N Megatron shard of the model (serving/engine.py).  Only rank 0 serves HTTP
and runs the :class:`~.engine.Scheduler`; every engine call it makes (prefill of one prompt or
of the prompts admitted together, one joint decode step) is first broadcast to the follower
ranks as a tiny command over a gloo control group, so all ranks issue the same sequence of collectives (RCCL for prefill /
logits, the one-shot IPC all-reduce for the decode step's per-layer reductions).  Sampling
happens on rank 0 only: the next step's tokens arrive with its command.

There is no counterpart in the reference (its serving story is a dashboard link to KServe);
the shape follows KServe's multi-GPU predictor (one pod, all GPUs of a node).
"""
from __future__ import annotations

from typing import List, Optional

import torch.distributed as dist

LEADER = 0   # global rank that serves HTTP


class TPLeaderEngine:
    """Rank-0 view of the engine: forwards each call to the followers, then runs it."""

    def __init__(self, engine, group=None):
        self.e = engine
        self.group = group

    def __getattr__(self, k):            # scratch, max_len, n_slots, cfg, ...
        return getattr(self.e, k)

    def _send(self, cmd: tuple):
        dist.broadcast_object_list([cmd], src=LEADER, group=self.group)

    def prefill(self, slot: int, tokens: List[int]):
        self._send(("prefill", int(slot), [int(t) for t in tokens]))
        return self.e.prefill(slot, tokens)

    def prefill_batch(self, slots: List[int], prompts: List[List[int]]):
        self._send(("prefill_batch", [int(s) for s in slots], [[int(t) for t in p] for p in prompts]))
        return self.e.prefill_batch(slots, prompts)

    def decode(self, tokens: List[int], slots: List[int], pos: List[int]):
        self._send(("decode", [int(t) for t in tokens], [int(s) for s in slots], [int(p) for p in pos]))
        return self.e.decode(tokens, slots, pos)

    def stop(self):
        self._send(("stop",))


def follower_loop(engine, group=None, max_commands: Optional[int] = None) -> int:
    """Ranks > 0: replay the leader's engine calls until it sends ``stop``.  Returns the
    number of commands executed."""
    n = 0
    while max_commands is None or n < max_commands:
        box = [None]
        dist.broadcast_object_list(box, src=LEADER, group=group)
        cmd = box[0]
        if cmd[0] == "stop":
            break
        if cmd[0] == "prefill":
            engine.prefill(cmd[1], cmd[2])
        elif cmd[0] == "prefill_batch":
            engine.prefill_batch(cmd[1], cmd[2])
        elif cmd[0] == "decode":
            engine.decode(cmd[1], cmd[2], cmd[3])
        else:
            raise ValueError(f"unknown TP predictor command {cmd[0]!r}")
        n += 1
    return n
