"""Context parallelism (Ulysses-style sequence/head all-to-all) for long-context training.

The ranks of one context-parallel group hold the same sequences, each rank a contiguous
1/cp block of every sequence's tokens.  Everything except attention is token-local: embedding,
norms, projections, MLP and the LM head run on the rank's own tokens; the weights are
replicated and their gradients are summed over the group like data parallelism (the trainer
uses the DP group as the CP group, so ZeRO-1 / the fp32 reduction apply unchanged).
Attention needs every token: before it, one all-to-all turns [own tokens, all heads] into
[all tokens, own 1/cp of the heads] (q, k and v head groups split alike, so GQA pairs stay
on one rank), RoPE and flash attention run on the full sequence for those heads, and the
inverse all-to-all brings the output back to [own tokens, all heads].  Backward mirrors it.

Per layer and direction that is two all-to-alls of [tokens/cp, width] -- bytes independent of
the number of ranks, unlike ring attention's cp-1 K/V passes -- and it needs Hkv % cp == 0
(Llama-3: 8 KV heads, so cp <= 8 = one MI355X node over xGMI)."""
from __future__ import annotations

from typing import List

import torch
import torch.distributed as dist


def to_heads(x: torch.Tensor, B: int, S_loc: int, widths: List[int], cp: int, group) -> torch.Tensor:
    """[B*S_loc, sum(widths)] (own tokens; column blocks ``widths``, e.g. q | k | v, each a run of
    heads) -> [B*S_loc*cp, sum(widths)/cp] (every token of the B sequences in order, this rank's
    1/cp of each block's heads)."""
    T = x.shape[0]
    parts, off = [[] for _ in range(cp)], 0
    for w in widths:
        assert w % cp == 0, (w, cp)
        step = w // cp
        for j in range(cp):
            parts[j].append(x[:, off + j * step:off + (j + 1) * step])
        off += w
    send = torch.stack([torch.cat(p, 1) for p in parts])          # [cp (dest), T, w/cp]
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)               # recv[i] = rank i's tokens
    wl = send.shape[-1]
    return recv.view(cp, B, S_loc, wl).transpose(0, 1).reshape(B * cp * S_loc, wl)


def to_tokens(y: torch.Tensor, B: int, S_loc: int, widths_local: List[int], cp: int, group) -> torch.Tensor:
    """Inverse of :func:`to_heads`: [B*S_loc*cp, sum(widths_local)] (all tokens, own head group)
    -> [B*S_loc, cp*sum(widths_local)] (own tokens, every head in the original column order)."""
    wl = y.shape[1]
    send = y.view(B, cp, S_loc, wl).transpose(0, 1).contiguous()  # [cp (dest token block), B, S_loc, wl]
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)               # recv[j] = own tokens, head group j
    recv = recv.view(cp, B * S_loc, wl)
    cols, off = [], 0
    for w in widths_local:
        cols.extend(recv[j, :, off:off + w] for j in range(cp))
        off += w
    return torch.cat(cols, 1)


def shard_tokens(t: torch.Tensor, cp: int, rank: int) -> torch.Tensor:
    """This rank's contiguous block of every sequence: [B, S] -> [B, S/cp]."""
    S = t.shape[1]
    assert S % cp == 0, (S, cp)
    n = S // cp
    return t[:, rank * n:(rank + 1) * n].contiguous()
