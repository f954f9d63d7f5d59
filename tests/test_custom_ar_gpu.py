"""One-shot IPC all-reduce (ops/csrc/custom_ar.hip) with 2, 4 and 8 ranks that share the single
GPU of the test box (gloo carries only the IPC-handle exchange; the data moves through the
peer-mapped uncached buffers).  On an 8-GPU node the same code runs one rank per GPU over xGMI;
the W = 4 / 8 instantiations (TP = 4 / 8 decode) run here first.  Expected: the kernel's defined
result, the fp32 sum of the bf16 inputs in rank order rounded once to bf16 -- bitwise."""
import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu


def _inp(n, it, r):
    g = torch.Generator(device="cpu").manual_seed(1000 * n + 10 * it + r)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _body(rank, world, n_list, iters):
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import OneShotAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = OneShotAllReduce(max_bytes=1 << 20, blocks=16, timeout_s=60.0)
    bad = []
    for n in n_list:
        for it in range(iters):
            y = car(_inp(n, it, rank).to("cuda:0"))
            torch.cuda.synchronize()
            acc = torch.zeros(n, dtype=torch.float32)
            for r in range(world):
                acc += _inp(n, it, r).float()
            if not torch.equal(y.cpu(), acc.to(torch.bfloat16)):
                bad.append((n, it))
    # the kernel inside a captured graph: the device-side epochs advance on every replay
    x = torch.full((4096,), float(rank + 1), device="cuda:0", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        car(x.clone())
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    dist.barrier()
    with torch.cuda.graph(graph):
        out = car(x.clone())          # in place on the clone: every replay starts from x
    dist.barrier()
    for _ in range(5):
        graph.replay()
    torch.cuda.synchronize()
    expect = world * (world + 1) / 2
    graph_ok = bool((out.float() == expect).all())
    err_flag = car.error()
    dist.barrier()
    car.close()
    return bad, graph_ok, err_flag


@pytest.mark.parametrize("world", [2, 4, 8])
def test_one_shot_allreduce_multirank_one_gpu(world):
    res = run_ranks(_body, world=world, args=([8, 4096, 65536, 262144], 3), timeout=300)
    for bad, graph_ok, err_flag in res:
        assert err_flag == 0
        assert graph_ok
        assert bad == [], bad


def _stall_body(rank, world):
    import time

    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import OneShotAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = OneShotAllReduce(max_bytes=1 << 20, blocks=4, timeout_s=1.0)
    x = torch.ones(4096, device="cuda:0", dtype=torch.bfloat16)
    car(x.clone())                        # both ranks: a healthy all-reduce first
    torch.cuda.synchronize()
    car.check()
    dist.barrier()
    raised = False
    if rank == 0:                          # rank 1 stalls: rank 0's kernel times out on it
        car(x.clone())
        torch.cuda.synchronize()
        try:
            car.check()
        except RuntimeError:
            raised = True
        # poisoned from now on, even though the error word was cleared by the read
        try:
            car.check()
            sticky = False
        except RuntimeError:
            sticky = True
    else:
        time.sleep(0.5)
        sticky = True
    dist.barrier()
    car.close()
    return rank, raised, sticky


def test_one_shot_allreduce_peer_stall_raises():
    """a stalled peer must surface as an error, not as silently wrong sums."""
    res = run_ranks(_stall_body, world=2, timeout=240)
    (r0, raised0, sticky0), _ = res
    assert r0 == 0 and raised0 and sticky0
