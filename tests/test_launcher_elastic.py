"""kfamd-launch elastic membership, driven directly (3 agents on this host, 1 worker each, gloo):

* a restarted (replacement) agent that re-joins while the group still runs must never be closed
  into a world of its own -- rounds need node 0, whose rank 0 hosts the TCPStore -- and the
  running agents re-join for it at once (membership change, not a used restart);
* losing node 0, which hosts the rendezvous server, is survived when a replacement node-0 agent
  comes back (restartPolicy OnFailure / ExitCode): the survivors re-join its new server;
* with no replacement the survivors give up after the rendezvous timeout (restartPolicy Never).
"""
import json
import os
import signal
import socket
import subprocess
import sys
import time

import pytest

from service_account_auth_improvements_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import datetime, json, os, sys, time
import torch, torch.distributed as dist
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=20))
r, w = dist.get_rank(), dist.get_world_size()
with open(sys.argv[1], "a") as f:
    f.write(json.dumps({"round": int(os.environ["KFAMD_RDZV_ROUND"]), "rank": r, "world": w,
                        "node": int(os.environ["NODE_RANK"]), "agent": os.environ["AGENT_TAG"]}) + "\n")
for i in range(int(sys.argv[2])):
    t = torch.ones(1)
    dist.all_reduce(t)
    assert int(t.item()) == w, (t, w)
    time.sleep(float(sys.argv[3]))      # a compute phase: peers notice a lost rank only at the next collective
dist.destroy_process_group()
"""


def _free_port_pair():
    while True:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p < 65000:
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", p + 1))
                return p
            except OSError:
                continue
            finally:
                t.close()


class Agents:
    def __init__(self, tmp_path, nnodes="1:3", iters=60, last_call=1.0, rdzv_timeout=60.0, step_s=0.1,
                 grace=3.0, worker=WORKER):
        self.exe = native.binary("kfamd_launch")
        self.out = tmp_path / "records.jsonl"
        self.script = tmp_path / "worker.py"
        self.script.write_text(worker)
        self.grace = grace
        self.port = _free_port_pair()
        self.nnodes, self.iters, self.last_call, self.rdzv_timeout = nnodes, iters, last_call, rdzv_timeout
        self.step_s = step_s
        self.logs = tmp_path
        self.procs = {}

    def start(self, node: int, tag: str, **extra_env):
        env = dict(os.environ, AGENT_TAG=tag, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **extra_env)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        cmd = [self.exe, "--nnodes", self.nnodes, "--node-rank", str(node), "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(self.port), "--max-restarts", "3",
               "--rdzv-last-call", str(self.last_call), "--rdzv-timeout", str(self.rdzv_timeout), "--grace", str(self.grace),
               "--", sys.executable, str(self.script), str(self.out), str(self.iters), str(self.step_s)]
        log = open(self.logs / f"agent_{tag}.log", "w")
        self.procs[tag] = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT)
        return self.procs[tag]

    def records(self):
        return [json.loads(x) for x in self.out.read_text().splitlines()] if self.out.exists() else []

    def wait_records(self, pred, timeout=90):
        deadline = time.time() + timeout
        while time.time() < deadline:
            if pred(self.records()):
                return True
            time.sleep(0.2)
        return False

    def wait_all(self, tags, timeout=120):
        deadline = time.time() + timeout
        rcs = {}
        for t in tags:
            try:
                rcs[t] = self.procs[t].wait(timeout=max(1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                rcs[t] = None
        return rcs

    def log(self, tag, full: bool = False):
        text = (self.logs / f"agent_{tag}.log").read_text()
        return text if full else text[-3000:]

    def stop(self):
        for p in self.procs.values():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in self.procs.values():
            try:
                p.wait(timeout=15)
            except subprocess.TimeoutExpired:
                p.kill()


@pytest.mark.slow
def test_replacement_agent_joins_the_running_group_never_a_world_of_its_own(tmp_path):
    """minReplicas 1, the split-world case: node 2 stops responding (its worker frozen, its agent
    gone) and a replacement node-2 agent starts while the survivors are still blocked in a
    collective with the frozen rank (as in an RCCL timeout, minutes).  Before the fix the server
    closed a round {2} after the last-call period and the replacement ran as rank 0 of a world
    of 1 against the running group's MASTER_PORT.  Now its round waits for node 0, the running
    agents see it waiting, stop their workers without using a restart, and the job finishes at
    world 3 with every agent exiting 0."""
    import psutil
    ag = Agents(tmp_path, nnodes="1:3", iters=60)
    frozen = None
    try:
        for n in range(3):
            ag.start(n, f"n{n}")
        assert ag.wait_records(lambda r: len([x for x in r if x["world"] == 3]) >= 3), \
            [ag.log(f"n{n}") for n in range(3)]
        frozen = psutil.Process(ag.procs["n2"].pid).children()[0]
        frozen.suspend()                                 # node 2 hangs: its sockets stay open
        ag.procs["n2"].kill()                            # its agent is gone (the pod is replaced)
        ag.procs["n2"].wait(timeout=20)
        ag.start(2, "n2b")                               # ...and the replacement pod comes up
        rcs = ag.wait_all(["n0", "n1", "n2b"], timeout=150)
        logs = {t: ag.log(t) for t in ("n0", "n1", "n2b")}
        assert rcs == {"n0": 0, "n1": 0, "n2b": 0}, (rcs, logs)
        rep = [x for x in ag.records() if x["agent"] == "n2b"]
        assert rep and all(x["world"] == 3 and x["rank"] == 2 for x in rep), (ag.records(), logs)
        # the survivors re-joined for the replacement: the last round is one world of all three
        last = max(x["round"] for x in ag.records())
        assert sorted(x["agent"] for x in ag.records() if x["round"] == last) == ["n0", "n1", "n2b"]
        full = {t: ag.log(t, full=True) for t in ("n0", "n1")}    # the workers' warnings can push it out of the tail
        assert "membership change" in full["n0"] and "membership change" in full["n1"], logs
        assert "restarts used" not in full["n0"] + full["n1"]
    finally:
        if frozen is not None:
            try:
                frozen.kill()
            except psutil.Error:
                pass
        ag.stop()


@pytest.mark.slow
def test_losing_node0_is_survived_when_its_replacement_rehosts_the_rendezvous(tmp_path):
    """Node 0 hosts the rendezvous server and rank 0's TCPStore.  Its agent is stopped and a
    replacement node-0 agent starts (a recreated el-worker-0 pod): the survivors' workers fail,
    their agents reach the replacement's new server, and all three finish together."""
    ag = Agents(tmp_path, nnodes="2:3", iters=60)
    try:
        for n in range(3):
            ag.start(n, f"n{n}")
        assert ag.wait_records(lambda r: len([x for x in r if x["world"] == 3]) >= 3), \
            [ag.log(f"n{n}") for n in range(3)]
        ag.procs["n0"].send_signal(signal.SIGTERM)
        ag.procs["n0"].wait(timeout=20)
        ag.start(0, "n0b")
        rcs = ag.wait_all(["n0b", "n1", "n2"], timeout=150)
        logs = {t: ag.log(t) for t in ("n0b", "n1", "n2")}
        assert rcs == {"n0b": 0, "n1": 0, "n2": 0}, (rcs, logs)
        after = [x for x in ag.records() if x["agent"] == "n0b"]
        assert after and after[-1]["world"] == 3 and after[-1]["rank"] == 0, (ag.records(), logs)
    finally:
        ag.stop()


@pytest.mark.slow
def test_losing_node0_without_replacement_fails_after_the_rendezvous_timeout(tmp_path):
    """restartPolicy Never: nothing re-hosts the rendezvous, so the survivors exit 3 once
    --rdzv-timeout (elasticPolicy rdzvConf join_timeout) has passed, instead of hanging."""
    ag = Agents(tmp_path, nnodes="1:3", iters=200, rdzv_timeout=8.0)
    try:
        for n in range(3):
            ag.start(n, f"n{n}")
        assert ag.wait_records(lambda r: len([x for x in r if x["world"] == 3]) >= 3), \
            [ag.log(f"n{n}") for n in range(3)]
        t0 = time.time()
        ag.procs["n0"].send_signal(signal.SIGTERM)
        rcs = ag.wait_all(["n1", "n2"], timeout=90)
        assert rcs == {"n1": 3, "n2": 3}, (rcs, ag.log("n1"), ag.log("n2"))
        assert time.time() - t0 < 60
    finally:
        ag.stop()


SLOW_EXIT_WORKER = r"""
import datetime, json, os, signal, sys, time
import torch, torch.distributed as dist
node, rnd = int(os.environ["NODE_RANK"]), int(os.environ["KFAMD_RDZV_ROUND"])
delay = float(os.environ.get("EXIT_DELAY", "0"))
def on_term(*_):                 # a GPU worker tearing down (HBM release, RCCL abort) takes a while
    time.sleep(delay)
    os._exit(143)
signal.signal(signal.SIGTERM, on_term)
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
r, w = dist.get_rank(), dist.get_world_size()
with open(sys.argv[1], "a") as f:
    f.write(json.dumps({"round": rnd, "rank": r, "world": w, "node": node, "agent": os.environ["AGENT_TAG"]}) + "\n")
for i in range(int(sys.argv[2])):
    if node == 2 and rnd == 1 and i == 5:
        os._exit(1)              # node 2's worker crashes once
    if i == 0 or i == int(sys.argv[2]) - 1:
        t = torch.ones(1)        # collectives at the ends only: in between a long compute phase,
        dist.all_reduce(t)       # so the peers learn of the crash from their agents' SIGTERM
    time.sleep(float(sys.argv[3]))
dist.destroy_process_group()
"""


@pytest.mark.slow
def test_slowly_exiting_workers_do_not_miss_the_restart_round(tmp_path):
    """on a membership change an agent stops its workers (SIGTERM, up to --grace)
    before it re-joins.  Node 1's worker takes 3 s to exit, longer than the 1 s last-call period:
    the server must wait for the previous round's members (up to grace + last call), so the
    restart round is ONE world of all three -- not a world {0, 2} closed without node 1 and
    then a second, free restart of everyone when node 1's late JOIN arrives."""
    ag = Agents(tmp_path, nnodes="2:3", iters=40, last_call=1.0, grace=6.0, worker=SLOW_EXIT_WORKER)
    try:
        ag.start(0, "n0")
        ag.start(1, "n1", EXIT_DELAY="3.0")
        ag.start(2, "n2")
        rcs = ag.wait_all(["n0", "n1", "n2"], timeout=150)
        logs = {t: ag.log(t) for t in ("n0", "n1", "n2")}
        assert rcs == {"n0": 0, "n1": 0, "n2": 0}, (rcs, logs)
        rounds = {}
        for x in ag.records():
            rounds.setdefault(x["round"], set()).add((x["node"], x["world"]))
        assert sorted(rounds) == [1, 2], (rounds, logs)            # exactly one restart round
        assert rounds[2] == {(0, 3), (1, 3), (2, 3)}, (rounds, logs)
    finally:
        ag.stop()
