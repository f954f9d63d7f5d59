"""Native (C++) runtime pieces: the per-node launcher / rendezvous agent.

``build_native()`` compiles every ``native/src/*.cpp`` into an executable under
``native/bin/`` (incremental, content-hashed), mirroring how the reference ships its
control-plane binaries as compiled artefacts.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "src"
BIN = HERE / "bin"


def build_native(force: bool = False) -> list:
    out = []
    if not SRC.exists():
        return out
    BIN.mkdir(exist_ok=True)
    for src in sorted(SRC.glob("*.cpp")):
        exe = BIN / src.stem
        stamp = BIN / (src.stem + ".stamp")
        h = hashlib.sha256(src.read_bytes()).hexdigest()[:16]
        if not force and exe.exists() and stamp.exists() and stamp.read_text() == h:
            out.append(exe)
            continue
        cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-pthread", str(src), "-o", str(exe)]
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"native build failed: {' '.join(cmd)}\n{p.stderr}")
        stamp.write_text(h)
        out.append(exe)
    return out


def binary(name: str) -> str:
    exe = BIN / name
    if not exe.exists():
        build_native()
    return str(exe)
