"""Per-rank progress marks and a no-progress watchdog for multi-rank GPU runs.

A hung collective (one rank skipped it, a peer died, a link went down) does not raise: every
other rank's host thread blocks in the next ``wait()`` / device synchronize until the process
group's timeout, and a run killed from outside at that point leaves no record of where it
stopped.  The runtime therefore marks what it is doing -- cheaply, one tuple assignment per
mark -- at its launch points (step boundaries, each DP bucket's collective, the ZeRO-1 parameter
gathers, pipeline hand-offs), and :class:`Watchdog` turns "no mark for ``timeout_s``" into a
diagnostic JSON line naming the last mark and a non-zero exit of this process (``os._exit``;
the launcher then tears the other ranks down).  The reference has no data plane and no
counterpart (SURVEY.md §5 "Failure detection": rank-failure detection is a [NS] requirement).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Callable, Optional

_last = (time.monotonic(), "start", None)
_count = 0


def mark(phase: str, detail: Optional[str] = None) -> None:
    """Record that this rank reached ``phase`` (``detail``: bucket / collective / step)."""
    global _last, _count
    _last = (time.monotonic(), phase, detail)
    _count += 1


def last() -> dict:
    ts, phase, detail = _last
    return {"phase": phase, "detail": detail, "idle_s": round(time.monotonic() - ts, 1), "marks": _count}


class Watchdog:
    """Daemon thread: when no :func:`mark` arrives for ``timeout_s`` seconds it writes
    ``report()`` merged with the last mark as one JSON line (stdout on the reporting rank,
    stderr elsewhere) and ends the process with ``exit_code``."""

    def __init__(self, timeout_s: float, report: Callable[[], dict], to_stdout: bool,
                 exit_code: int = 3, poll_s: float = 0.5):
        self.timeout_s = float(timeout_s)
        self.report = report
        self.to_stdout = to_stdout
        self.exit_code = exit_code
        self.poll_s = poll_s
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "Watchdog":
        mark("watchdog armed")
        self._thread = threading.Thread(target=self._run, name="kfamd-progress-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            info = last()
            if info["idle_s"] < self.timeout_s:
                continue
            rec = dict(self.report())
            rec["error"] = f"no progress for {self.timeout_s:.0f} s"
            rec["stopped_at"] = info
            line = json.dumps(rec)
            stream = sys.stdout if self.to_stdout else sys.stderr
            try:
                stream.write(line + "\n")
                stream.flush()
                if self.to_stdout:
                    sys.stderr.write(line + "\n")
                    sys.stderr.flush()
            finally:
                os._exit(self.exit_code)
