"""ASan + UBSan runs of the native host code (VERDICT r1 hygiene: "a CPU ASan+UBSan build and
run of native/src/kfamd_launch.cpp and the host side of ops/csrc/bindings.cpp").

* kfamd_launch (g++ -fsanitize=address,undefined, leak checking on): single node, two-node
  rendezvous over localhost, failure fan-out, heartbeat timeout, restart, SIGTERM.
* ops_host_check (bindings.cpp + every .hip launcher, host pass instrumented, libtorch):
  argument validation through the dispatcher on the CPU; with a GPU, real launches of every
  op against fp32 ATen references.

Any sanitizer report aborts the binary (halt_on_error) and is also searched for in stderr.
"""
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from service_account_auth_improvements_amd.native import sanitize

REPORTS = ("AddressSanitizer", "LeakSanitizer", "runtime error:", "UndefinedBehaviorSanitizer")


@pytest.fixture(scope="module")
def launch():
    return str(sanitize.build_launch())


def _env(extra=None):
    e = dict(os.environ)
    e.update(sanitize.ASAN_ENV)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PET_NNODES",
              "PET_NODE_RANK", "PET_NPROC_PER_NODE", "PET_MASTER_ADDR", "PET_MASTER_PORT"):
        e.pop(k, None)
    e.update(extra or {})
    return e


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _clean(err: str):
    for r in REPORTS:
        assert r not in err, err


def _run(args, timeout=60, env=None):
    p = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env or _env())
    _clean(p.stderr)
    return p


def test_launch_single_node_env(launch, tmp_path):
    mp = _port()
    p = _run([launch, "--nproc-per-node", "3", "--master-port", str(mp), "--",
              "sh", "-c", f'echo "$RANK $LOCAL_RANK $WORLD_SIZE $MASTER_PORT $HSA_ENABLE_IPC_MODE_LEGACY" '
                          f'> {tmp_path}/r$RANK'])
    assert p.returncode == 0, p.stderr
    got = sorted((tmp_path / f"r{r}").read_text().split() for r in range(3))
    assert got == [[str(r), str(r), "3", str(mp), "0"] for r in range(3)]


def test_launch_two_node_rendezvous(launch, tmp_path):
    mp = _port()
    common = ["--nnodes", "2", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
              "--master-port", str(mp), "--rdzv-port", str(_port()), "--rdzv-timeout", "30", "--",
              "sh", "-c", f'echo "$RANK $WORLD_SIZE $NODE_RANK" > {tmp_path}/r$RANK']
    procs = [subprocess.Popen([launch, "--node-rank", str(n), *common], stderr=subprocess.PIPE,
                              text=True, env=_env()) for n in (1, 0)]
    for pr in procs:
        _, err = pr.communicate(timeout=60)
        _clean(err)
        assert pr.returncode == 0, err
    rows = sorted(tuple((tmp_path / f"r{r}").read_text().split()) for r in range(4))
    assert [r[:2] for r in rows] == [(str(r), "4") for r in range(4)]
    assert {r[2] for r in rows} == {"0", "1"}


def test_launch_failure_fans_out(launch):
    t0 = time.time()
    p = _run([launch, "--nproc-per-node", "2", "--grace", "2", "--master-port", str(_port()), "--",
              "sh", "-c", 'if [ "$LOCAL_RANK" = 1 ]; then exit 7; fi; sleep 30'])
    assert p.returncode == 7, p.stderr
    assert time.time() - t0 < 20          # the sleeping sibling was terminated, not awaited


def test_launch_heartbeat_timeout(launch):
    p = _run([launch, "--nproc-per-node", "1", "--heartbeat-timeout", "0.5", "--grace", "1",
              "--master-port", str(_port()), "--", "sh", "-c", "touch $KFAMD_HEARTBEAT_FILE; sleep 30"])
    assert p.returncode == 124, p.stderr
    assert "missed its heartbeat" in p.stderr


def test_launch_restart_then_succeed(launch, tmp_path):
    marker = tmp_path / "failed_once"
    p = _run([launch, "--nproc-per-node", "2", "--max-restarts", "2", "--grace", "1",
              "--master-port", str(_port()), "--", "sh", "-c",
              f'if [ "$RANK" = 0 ] && [ ! -e {marker} ]; then touch {marker}; exit 3; fi; '
              f'echo $KFAMD_RDZV_ROUND > {tmp_path}/round$RANK'])
    assert p.returncode == 0, p.stderr
    assert (tmp_path / "round0").read_text().strip() == "2"
    assert "restarting workers" in p.stderr


def test_launch_sigterm_stops_workers(launch, tmp_path):
    pr = subprocess.Popen([launch, "--nproc-per-node", "2", "--grace", "1", "--master-port", str(_port()),
                           "--", "sh", "-c", f"echo $$ > {tmp_path}/pid$LOCAL_RANK; sleep 60"],
                          stderr=subprocess.PIPE, text=True, env=_env())
    deadline = time.time() + 20
    while time.time() < deadline and not all((tmp_path / f"pid{i}").exists() for i in range(2)):
        time.sleep(0.05)
    time.sleep(0.2)
    pr.send_signal(signal.SIGTERM)
    _, err = pr.communicate(timeout=30)
    _clean(err)
    assert pr.returncode == 143, err
    for i in range(2):
        pid = int((tmp_path / f"pid{i}").read_text())
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)


def test_launch_rejects_bad_args(launch):
    p = _run([launch, "--nnodes", "2", "--node-rank", "5", "--", "true"])
    assert p.returncode == 2


@pytest.fixture(scope="module")
def ops_check():
    return str(sanitize.build_ops_check())


def _ops_env():
    e = dict(os.environ)
    e.update(sanitize.OPS_ASAN_ENV)
    return e


def test_ops_host_validation_sanitized(ops_check):
    p = subprocess.run([ops_check], capture_output=True, text=True, timeout=300, env=_ops_env(), cwd="/tmp")
    _clean(p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 failed" in p.stdout


@pytest.mark.gpu
def test_ops_host_sanitized_gpu_launches(ops_check):
    p = subprocess.run([ops_check, "--gpu"], capture_output=True, text=True, timeout=300, env=_ops_env(),
                       cwd="/tmp")
    sys.stdout.write(p.stdout)
    _clean(p.stderr)
    assert p.returncode == 0, p.stdout + p.stderr[-4000:]
    assert "0 failed" in p.stdout and "PASS flash_bwd dk" in p.stdout
