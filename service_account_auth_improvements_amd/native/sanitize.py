"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the native host code (SURVEY §5
"Race detection / sanitizers"; VERDICT r1 hygiene item).

Two instrumented binaries go to ``native/bin/san/``:

* ``kfamd_launch`` -- the per-node launcher/rendezvous agent (``native/src/kfamd_launch.cpp``),
  g++ with ``-fsanitize=address,undefined``; leak checking stays on.  ``tests/test_native_sanitize.py``
  runs it through single-node, two-node rendezvous, failure fan-out, heartbeat and restart
  scenarios on the CPU.
* ``ops_host_check`` -- ``ops/csrc/bindings.cpp`` and every ``ops/csrc/*.hip`` launcher with the
  sanitizers on the HOST side only (device code is the ordinary gfx950 code), linked with
  libtorch and driven through the dispatcher by ``native/sanitize/ops_host_check.cpp``.  The
  validation half runs on the CPU; ``--gpu`` adds real launches checked against fp32 ATen
  references (``tests/test_native_sanitize.py`` GPU test).  GPU-side sanitizers are not used.

Incremental like the other builds (content hash of sources + flags).
Usage: ``python -m service_account_auth_improvements_amd.native.sanitize [--force]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
CSRC = PKG / "ops" / "csrc"
OUT = HERE / "bin" / "san"
TMP = OUT / "obj"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KFAMD_ARCH", "gfx950")

# UBSan minus the checks that misfire on uninstrumented libtorch frames (vptr needs RTTI of
# every dynamic type; -fsanitize=function flags torch's boxed-kernel function-pointer casts).
UB_OFF = ["-fno-sanitize=vptr", "-fno-sanitize=function", "-fno-sanitize-recover=all"]

# Environment for running the instrumented binaries: abort on the first report.
ASAN_ENV = {
    "ASAN_OPTIONS": "halt_on_error=1:abort_on_error=0:detect_leaks=1:strict_string_checks=1:"
                    "detect_stack_use_after_return=1:check_initialization_order=1",
    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
}
# libtorch keeps process-lifetime singletons that LSan would report at exit, and the ROCm
# runtime maps device apertures in the range ASan would otherwise protect.
OPS_ASAN_ENV = {
    "ASAN_OPTIONS": "halt_on_error=1:abort_on_error=0:detect_leaks=0:protect_shadow_gap=0:"
                    "alloc_dealloc_mismatch=0",
    "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
}


def _digest(files, flags) -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(str(f).encode())
        h.update(Path(f).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"sanitizer build failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")


def _fresh(exe: Path, digest: str, force: bool) -> bool:
    stamp = exe.with_suffix(".stamp")
    return not force and exe.exists() and stamp.exists() and stamp.read_text() == digest


def build_launch(force: bool = False) -> Path:
    src = HERE / "src" / "kfamd_launch.cpp"
    exe = OUT / "kfamd_launch"
    flags = ["-O1", "-g", "-std=c++17", "-Wall", "-pthread", "-fno-omit-frame-pointer",
             "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]
    dg = _digest([src], flags)
    if _fresh(exe, dg, force):
        return exe
    OUT.mkdir(parents=True, exist_ok=True)
    _run(["g++", *flags, str(src), "-o", str(exe)])
    exe.with_suffix(".stamp").write_text(dg)
    return exe


def build_ops_check(force: bool = False, jobs: int | None = None) -> Path:
    import torch
    import torch.utils.cpp_extension as ce

    from ..ops._build import FILE_FLAGS

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    base = ["-O1", "-g", "-std=c++17", "-fPIC", "-fno-omit-frame-pointer",
            "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-Wno-unused-result", "-Wno-deprecated-declarations"]
    # .hip sources: device code for gfx950 as usual, sanitizers on the host pass only
    hip_flags = base + [f"--offload-arch={ARCH}", "-ffp-contract=fast", "-munsafe-fp-atomics",
                        "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                        *[x for f in UB_OFF for x in ("-Xarch_host", f)]]
    # host-only C++ (bindings + harness): no device pass at all
    cpp_flags = base + [f"-I{p}" for p in inc] + [
        "-DTORCH_EXTENSION_NAME=_kfamd_ops", "-DHIP_ENABLE_WARP_SYNC_BUILTINS=1",
        "-fsanitize=address", "-fsanitize=undefined", "-fno-gpu-sanitize", *UB_OFF]
    link = ["-fsanitize=address", "-fsanitize=undefined", "-fno-gpu-sanitize", f"--offload-arch={ARCH}",
            f"-L{lib}", f"-Wl,-rpath,{lib}", "-Wl,--no-as-needed", "-ltorch_hip", "-lc10_hip",
            "-ltorch", "-ltorch_cpu", "-lc10", "-Wl,--as-needed", "-lamdhip64", "-pthread"]
    hips = sorted(CSRC.glob("*.hip"))
    cpps = [CSRC / "bindings.cpp", HERE / "sanitize" / "ops_host_check.cpp"]
    exe = OUT / "ops_host_check"
    dg = _digest(hips + cpps + sorted(CSRC.glob("*.h")),
                 hip_flags + cpp_flags + link + [f"{k}:{v}" for k, v in sorted(FILE_FLAGS.items())])
    if _fresh(exe, dg, force):
        return exe
    TMP.mkdir(parents=True, exist_ok=True)
    cmds, objs = [], []
    for s in hips:
        o = TMP / (s.stem + ".o")
        objs.append(o)
        cmds.append([HIPCC, *hip_flags, *FILE_FLAGS.get(s.name, []), "-c", str(s), "-o", str(o)])
    for s in cpps:
        o = TMP / (s.stem + ".o")
        objs.append(o)
        cmds.append([HIPCC, "-x", "c++", *cpp_flags, "-c", str(s), "-o", str(o)])
    with cf.ThreadPoolExecutor(max_workers=jobs or min(8, os.cpu_count() or 4)) as ex:
        list(ex.map(_run, cmds))
    _run([HIPCC, *map(str, objs), *link, "-o", str(exe)])
    exe.with_suffix(".stamp").write_text(dg)
    return exe


def build_all(force: bool = False) -> list:
    return [build_launch(force), build_ops_check(force)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    for p in build_all(a.force):
        print(p)


if __name__ == "__main__":
    main()
