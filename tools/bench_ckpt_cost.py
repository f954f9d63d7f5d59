"""Step-time cost of the worker's asynchronous periodic checkpoint on the GPU.

Runs the PyTorchJob worker (runtime/train_entry.py) at the bench configuration (Llama-3-8B,
S 8192, micro-batch 4, ZeRO-1) with ``--ckpt-dir DIR --save-every K`` and reads its own events:
every step's device time (``step_s``, end event to end event), the steps whose optimizer update
waited for a snapshot (the step after each save), and each save's publish time (snapshot ->
every file written and fsynced -> ``latest`` replaced).  One JSON line:

  {"steady_ms": ..., "after_save_ms": [...], "save_cost_ms": ..., "publish_s": [...], "state_gb": ...}

  python tools/bench_ckpt_cost.py --dir /tmp/ckpt [--steps 14] [--save-every 5] [--layers N]

The checkpoint holds the bf16 parameters and the fp32 master + AdamW moments (112 GB at 8B and
one data-parallel rank): DIR needs that much free space, and the host the same in pinned memory.
"""
import argparse
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--steps", type=int, default=14)
    ap.add_argument("--save-every", type=int, default=5)
    ap.add_argument("--micro-batch", type=int, default=4)
    ap.add_argument("--layers", type=int, default=None, help="smaller state (the cost scales with it)")
    a = ap.parse_args()
    ev = os.path.join(tempfile.mkdtemp(prefix="ckpt-cost-"), "events.jsonl")
    shutil.rmtree(a.dir, ignore_errors=True)
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", "llama3-8b",
           "--seq-len", "8192", "--micro-batch", str(a.micro_batch), "--zero1", "--steps", str(a.steps),
           "--ckpt-dir", a.dir, "--save-every", str(a.save_every), "--keep-checkpoints", "1"]
    if a.layers:
        cmd += ["--layers", str(a.layers)]
    try:
        subprocess.run(cmd, check=True, env=dict(os.environ, KFAMD_EVENTS_FILE=ev, PYTHONPATH=ROOT), cwd=ROOT,
                       stdout=subprocess.DEVNULL)
        size = sum(os.path.getsize(os.path.join(dp, f)) for dp, _, fs in os.walk(a.dir) for f in fs)
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)
    with open(ev) as f:
        recs = [json.loads(x) for x in f if x.strip()]
    step_s = {r["step"]: r["step_s"] for r in recs if r["event"] == "step" and "step_s" in r}
    saves = [r["step"] for r in recs if r["event"] == "checkpoint_queued"]
    # the save after step k-1 (published as "step k") is snapshotted while step k runs; step k's
    # optimizer update waits for the copy
    hit = {s for s in saves}
    steady = [v for k, v in step_s.items() if k >= 2 and k not in hit]
    after = [step_s[k] for k in sorted(hit) if k in step_s]
    med = statistics.median(steady)
    out = {"steady_ms": round(med * 1e3, 1), "after_save_ms": [round(x * 1e3, 1) for x in after],
           "save_cost_ms": round((statistics.mean(after) - med) * 1e3, 1) if after else None,
           "publish_s": [r["seconds"] for r in recs if r["event"] == "checkpoint_published"],
           "saves": saves, "state_gb": round(size / 1e9, 1), "layers": a.layers or 32}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
