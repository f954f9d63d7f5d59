"""The framework's training step against plain PyTorch: the Trainer (explicit forward/backward,
flat buffers, FlatAdamW, clipping) and the standard nn.Module + autograd + torch.optim.AdamW
model of tools/bench_torch_baseline.py start from the same weights and must produce the same
loss trajectory over several steps (tools/compare_torch_trajectory.py runs the same check on
the GPU kernels)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_training_trajectory_matches_plain_pytorch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "compare_torch_trajectory.py"), "tiny", "2", "128",
                        "8"], capture_output=True, text=True, timeout=600, cwd="/tmp",
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stderr[-2000:]
    last = r.stdout.strip().splitlines()[-1]
    worst = float(last.rsplit(" ", 1)[1])
    assert worst < 2e-3, r.stdout
    steps = [l.split() for l in r.stdout.splitlines() if l.startswith("step")]
    assert len(steps) == 8 and float(steps[-1][3]) < float(steps[0][3])      # it learns
