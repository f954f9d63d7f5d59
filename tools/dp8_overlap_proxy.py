"""One-GPU proxy for the N = 8 data-parallel overlap cost.

At N = 8 the ZeRO-1 step (bench.py's plan) moves, per GPU and step, the bucketed all-to-all of
the bf16 gradients (7/8 of 16 GB out and in, launched bucket by bucket while backward runs) and
the bf16 parameter all-gather (7/8 of 16 GB in, launched after the optimizer, waited for bucket
by bucket by the next forward): ~28 GB.  RCCL moves it with one workgroup per channel, and those
workgroups sit on the CUs the GEMMs and attention need.  The one-rank RCCL rehearsal
(``bench.py --force-collectives``) turns the all-to-all into a local copy and shows none of that.

This tool runs the real full-size 1-GPU training step (Llama-3-8B, S 8192, micro-batch 4, the
bench's config) with ``GradReducer.traffic_proxy`` set: at every bucket launch (the moment the
bucket's gradients are final on the compute stream) it launches, on a side stream,
tools/kbench/proxy_traffic.hip with C workgroups that hold their CUs for as long as the bucket's
all-to-all takes at the modelled xGMI rate, copying the bucket's bytes through HBM as they go;
``finish()`` makes the optimizer wait for them (it needs the reduced gradients), and the
parameter gather is modelled the same way after the optimizer.  C = 0 (no proxy), 8, 16, 32, 64.

The predicted N = 8 step is the proxy step plus the exposed tail that cannot overlap: the last
bucket's all-to-all after backward and the first bucket's gather before the first forward layer.
Output: one JSON line per configuration and a summary line -> profiles/dp8_overlap_proxy.md.

  python tools/dp8_overlap_proxy.py [--channels 0,8,16,32,64] [--link-gbs 64] [--steps 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

WORLD = 8


class Proxy:
    def __init__(self, lib, channels: int, rate_gbs: float, max_bytes: int):
        self.lib, self.channels, self.rate = lib, channels, rate_gbs
        self.stream = torch.cuda.Stream()
        self.src = torch.empty(max_bytes, dtype=torch.uint8, device="cuda")
        self.dst = torch.empty(max_bytes, dtype=torch.uint8, device="cuda")
        self.bytes_moved = 0
        self.calls = 0

    def _launch(self, nbytes: int):
        q = 16 * self.channels
        n = (int(nbytes * (WORLD - 1) / WORLD) // q) * q
        if n <= 0:
            return
        ev = torch.cuda.Event()
        ev.record()                                   # the bucket is final on the compute stream
        self.stream.wait_event(ev)
        rc = self.lib.proxy_traffic(ctypes.c_void_p(self.src.data_ptr()), ctypes.c_void_p(self.dst.data_ptr()),
                                    ctypes.c_long(n), ctypes.c_int(self.channels), ctypes.c_double(self.rate),
                                    ctypes.c_void_p(self.stream.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"proxy_traffic rc={rc}")
        self.bytes_moved += n
        self.calls += 1

    def on_bucket(self, nbytes: int):
        self._launch(nbytes)

    def on_finish(self):
        torch.cuda.current_stream().wait_stream(self.stream)   # the optimizer reads reduced grads

    def on_gather(self, nbytes: int):
        self._launch(nbytes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", default="0,8,16,32,64,0")
    ap.add_argument("--link-gbs", type=float, default=64.0,
                    help="usable unidirectional GB/s per xGMI link; 7 links per GPU carry the all-to-all")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--layers", type=int, default=None, help="DEBUG ONLY")
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "kbench", "bin", "libproxy_traffic.so"))
    lib.proxy_traffic.restype = ctypes.c_int
    from service_account_auth_improvements_amd.ops import _build
    _build.build()
    from service_account_auth_improvements_amd.parallel.state import init_distributed
    from service_account_auth_improvements_amd.runtime.trainer import SyntheticData, TrainConfig, Trainer
    st = init_distributed(device="cuda")
    tcfg = TrainConfig(model="llama3-8b", seq_len=8192, micro_batch=a.micro_batch, zero1=True, n_layers=a.layers)
    tr = Trainer(tcfg, st)
    data = SyntheticData(tr.mcfg.vocab_size, a.micro_batch, 8192, st.device, seed=1)
    batches = [[data.next()] for _ in range(2)]
    bucket_bytes = max(b.hi - b.lo for bl in tr.reducer.buckets.values() for b in bl) * 2
    rate = 7 * a.link_gbs
    results = []
    proxies = {}
    # what C workgroups can move at all (unpaced, no training): below the modelled link rate the
    # proxy itself becomes the exposed communication, as an RCCL run with too few channels would
    unpaced = {}
    for ch in sorted({int(x) for x in a.channels.split(",") if int(x) > 0}):
        px = Proxy(lib, ch, 1e6, bucket_bytes)
        n = (bucket_bytes // (16 * ch)) * 16 * ch
        for _ in range(2):
            px._launch(n * WORLD // (WORLD - 1))
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(px.stream)
        for _ in range(5):
            px._launch(n * WORLD // (WORLD - 1))
        e1.record(px.stream)
        torch.cuda.synchronize()
        unpaced[ch] = round(5 * px.bytes_moved / 7 / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)
        del px
        print(json.dumps({"channels": ch, "unpaced_copy_gbs": unpaced[ch], "modelled_link_gbs": rate}), flush=True)
    for ch in [int(x) for x in a.channels.split(",")]:
        if ch > 0 and ch not in proxies:
            proxies[ch] = Proxy(lib, ch, rate, bucket_bytes)
        tr.reducer.traffic_proxy = proxies.get(ch)
        for i in range(a.warmup):
            tr.train_step(batches[i % 2])
        torch.cuda.synchronize()
        moved0 = proxies[ch].bytes_moved if ch else 0
        t0 = time.perf_counter()
        for i in range(a.steps):
            tr.train_step(batches[i % 2])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        rec = {"channels": ch, "ms_per_step": round(dt * 1e3, 2),
               "proxy_gb_per_step": round(((proxies[ch].bytes_moved - moved0) if ch else 0) / a.steps / 1e9, 2)}
        results.append(rec)
        print(json.dumps(rec), flush=True)
    tr.reducer.traffic_proxy = None
    base = [r["ms_per_step"] for r in results if r["channels"] == 0]
    t1 = sum(base) / len(base)
    bucket_s = bucket_bytes * (WORLD - 1) / WORLD / (rate * 1e9)
    tail_ms = 2 * bucket_s * 1e3                   # last a2a after backward + first gather before forward
    summary = {"baseline_ms": round(t1, 2), "baseline_spread_ms": round(max(base) - min(base), 2),
               "bucket_mb": bucket_bytes >> 20, "link_gbs": a.link_gbs, "modelled_a2a_ms_per_bucket": round(bucket_s * 1e3, 3),
               "exposed_tail_ms": round(tail_ms, 2), "predicted": {}}
    for r in results:
        if r["channels"]:
            t8 = r["ms_per_step"] + tail_ms
            summary["predicted"][str(r["channels"])] = {"unpaced_copy_gbs": unpaced.get(r["channels"]),
                                                        "slowdown_pct": round(100 * (r["ms_per_step"] / t1 - 1), 2),
                                                        "n8_ms_per_step": round(t8, 1),
                                                        "n8_efficiency": round(t1 / t8, 4)}
    print(json.dumps({"summary": summary}), flush=True)


if __name__ == "__main__":
    main()
