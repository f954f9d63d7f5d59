"""One-shot IPC all-reduce (ops/csrc/custom_ar.hip) vs a float64 sum, with two ranks that
share the single GPU of the test box (gloo carries only the IPC-handle exchange; the data
moves through the peer-mapped uncached buffers).  On an 8-GPU node the same code runs one
rank per GPU over xGMI."""
import pytest
import torch

from dist_util import run_ranks

pytestmark = pytest.mark.gpu


def _body(rank, world, n_list, iters):
    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import OneShotAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = OneShotAllReduce(max_bytes=1 << 20, blocks=16)
    errs = []
    for n in n_list:
        for it in range(iters):
            g = torch.Generator(device="cpu").manual_seed(1000 * n + 10 * it + rank)
            x = torch.randn(n, generator=g).to("cuda:0", torch.bfloat16)
            y = car(x)
            torch.cuda.synchronize()
            ref = torch.zeros(n, dtype=torch.float64)
            for r in range(world):
                gr = torch.Generator(device="cpu").manual_seed(1000 * n + 10 * it + r)
                ref += torch.randn(n, generator=gr).to(torch.bfloat16).double()
            errs.append(float((y.double().cpu() - ref).abs().max()))
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
    return max(errs), graph_ok, err_flag


def test_one_shot_allreduce_two_ranks_one_gpu():
    res = run_ranks(_body, world=2, args=([8, 4096, 65536, 262144], 3), timeout=240)
    for max_err, graph_ok, err_flag in res:
        assert err_flag == 0
        assert graph_ok
        assert max_err < 0.05, max_err     # bf16 output rounding of a 2-term sum


def _stall_body(rank, world):
    import time

    import torch.distributed as dist

    from service_account_auth_improvements_amd.parallel.custom_ar import OneShotAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = OneShotAllReduce(max_bytes=1 << 20, blocks=4)
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
