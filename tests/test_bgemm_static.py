"""Static guard for the batched-decode GEMM (ops/csrc/bgemm.hip), CPU only: its W operands are
loaded by inline asm outside hipcc's wait bookkeeping, so the compiled code must never read
such a register (a copy, a spill) before the MFMA that consumes it after the kernel's own
counted wait -- checked on the gfx950 assembly (tools/check_inflight_regs.py)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="needs hipcc")
def test_bgemm_asm_loads_are_only_read_by_their_mfma(capsys):
    import check_inflight_regs
    assert check_inflight_regs.main() == 0, capsys.readouterr().out
    out = capsys.readouterr().out
    # 4 row tilings x 1 / 2 W tiles per wave x plain / SwiGLU, every one free of unsafe reads
    lines = [x for x in out.splitlines() if "bgemm_kernel" in x]
    assert len(lines) == 16 and all("unsafe reads 0" in x for x in lines), out
