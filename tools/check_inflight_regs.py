"""Static check of a kernel's inline-asm register loads (ops/csrc/bgemm.hip): the W operands are
loaded by `global_load_dwordx4 ... nt` in inline asm, so hipcc does not track them and only the
kernel's own counted vmcnt waits protect them.  Each kernel body is scanned in text order with
the vmcnt queue modelled (every VMEM load queued, `s_waitcnt vmcnt(N)` retires all but the
newest N): any read of an asm-loaded register while its load is queued (a missing or short
wait, a copy, a spill) and any other write to it (hipcc reusing a register it thinks is free --
the load then lands on top of the new value) is reported.  Also reports scratch use.

    python tools/check_inflight_regs.py [source.hip] -> exit 1 on a finding
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "service_account_auth_improvements_amd", "ops", "csrc", "bgemm.hip")


def _regs(s):
    out = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", s):
        out |= set(range(int(a), int(b) + 1))
    for a in re.findall(r"(?<![\w\[:])v(\d+)\b", s):
        out.add(int(a))
    return out


def check_body(lines):
    """Linear scan with the vmcnt queue modelled in issue order: every VMEM load is queued, an
    `s_waitcnt vmcnt(N)` retires all but the newest N.  A read of an asm-loaded register while
    its load is queued, or any other write to it, is a hazard (the load lands later)."""
    queue, bad, consumers = [], [], 0          # queue: list of register sets (empty for non-asm loads)
    for i, ln in enumerate(lines):
        if not ln or ln[0] in ";.":
            continue
        m = re.search(r"s_waitcnt\b.*vmcnt\((\d+)\)", ln)
        if m:
            n = int(m.group(1))
            del queue[:max(0, len(queue) - n)]
            continue
        if ln.startswith("s_"):
            continue
        op, _, args = ln.partition(" ")
        parts = [p.strip() for p in args.split(",")]
        busy = set().union(*queue) if queue else set()
        stores = "store" in op or (op.startswith("ds_") and "write" in op)
        srcs = set()
        for p in parts[1:]:
            srcs |= _regs(p)
        if stores:
            srcs |= _regs(parts[0])
        dst = set() if stores else _regs(parts[0])
        asm_load = op == "global_load_dwordx4" and ln.endswith(" nt")
        if srcs & busy:
            bad.append((i, "read of an in-flight asm-load register: " + ln))
        elif op.startswith("v_mfma"):
            consumers += 1
        if dst & busy:
            bad.append((i, "write to an in-flight asm-load register: " + ln))
        if op.startswith(("global_load", "buffer_load", "global_atomic", "flat_load")):
            queue.append(dst if asm_load else set())
    return consumers, bad


def main(src=SRC):
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
                        "-S", "-I", os.path.dirname(src), src, "-o", asm], check=True, capture_output=True)
        text = open(asm).read()
    kernels = re.findall(r"^(_Z\w+):[^\n]*\n(.*?)s_endpgm", text, re.S | re.M)
    failures = 0
    for name, body in kernels:
        lines = [ln.strip() for ln in body.split("\n")]
        consumers, bad = check_body(lines)
        scratch = sum(1 for ln in lines if ln.startswith("scratch_") or ln.startswith("buffer_store_dword") and "off, s[0:3]" in ln)
        print(f"{name[:60]:60s} asm-load consumers {consumers:3d}  unsafe reads {len(bad)}  scratch ops {scratch}")
        for b in bad[:5]:
            print("    ", b)
        failures += len(bad) + scratch
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
