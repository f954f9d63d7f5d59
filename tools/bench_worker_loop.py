"""The PyTorchJob worker's steady-state step time next to bench.py's.

Runs the worker a PyTorchJob pod runs (``python -m service_account_auth_improvements_amd train``,
runtime/train_entry.py) for ``--steps`` steps at the bench's configuration (Llama-3-8B, S 8192,
micro-batch 4, ZeRO-1, fp32 gradient reduction), then ``bench.py`` on the same box, each in a
fresh process.  The worker's steady state is taken from its own ``step`` events: the device time
between consecutive steps' end events (``step_s``), median over the steps after ``--skip``, and
the host wall clock across the same steps.  One JSON line:

  {"worker_ms_per_step": ..., "worker_wall_ms_per_step": ..., "bench_ms_per_step": ..., "ratio": ...}

  python tools/bench_worker_loop.py [--steps 25] [--skip 5]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--micro-batch", type=int, default=4)
    a = ap.parse_args()
    ev = os.path.join(tempfile.mkdtemp(prefix="worker-loop-"), "events.jsonl")
    env = dict(os.environ, KFAMD_EVENTS_FILE=ev, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "service_account_auth_improvements_amd", "train", "--model", "llama3-8b",
           "--seq-len", "8192", "--micro-batch", str(a.micro_batch), "--zero1", "--steps", str(a.steps)]
    subprocess.run(cmd, check=True, env=env, cwd=ROOT, stdout=subprocess.DEVNULL)
    with open(ev) as f:
        recs = [json.loads(x) for x in f if x.strip()]
    steps = [r for r in recs if r["event"] == "step" and r["step"] >= a.skip]
    dev = statistics.median(r["step_s"] for r in steps if "step_s" in r) * 1e3
    wall = (steps[-1]["ts"] - steps[0]["ts"]) / (len(steps) - 1) * 1e3
    b = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                        "--crd-jobs", "0", "--micro-batch", str(a.micro_batch)],
                       check=True, env=dict(os.environ), cwd=ROOT, capture_output=True, text=True)
    rec = json.loads([x for x in b.stdout.splitlines() if x.startswith("{")][-1])
    out = {"worker_ms_per_step": round(dev, 2), "worker_wall_ms_per_step": round(wall, 2),
           "bench_ms_per_step": rec["ms_per_step"], "ratio_worker_over_bench": round(wall / rec["ms_per_step"], 4),
           "worker_steps_measured": len(steps), "config": rec["config"]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
