"""In-tree build of the gfx950 HIP kernels into ``ops/_kfamd_ops.so``.

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an object
file; ``csrc/bindings.cpp`` (the only TU that includes libtorch) registers the
``torch.ops.kfamd.*`` operators; the objects are linked into one shared library that is
loaded with ``torch.ops.load_library``.  The build is incremental (content hash of the
sources + flags) so importing the package on a box that already has the ``.so`` costs
nothing, and it runs on a CPU-only machine (hipcc cross-compiles for gfx950).

Usage: ``python -m service_account_auth_improvements_amd.ops._build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build_tmp"
LIB_NAME = "_kfamd_ops.so"
LIB_PATH = HERE / LIB_NAME
ARCH = os.environ.get("KFAMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _flags():
    inc, lib, abi = _torch_paths()
    common = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-Wno-unused-result", "-Wno-deprecated-declarations",
    ]
    kernel = common + ["-ffp-contract=fast", "-munsafe-fp-atomics"]
    binding = common + [f"-I{p}" for p in inc] + ["-DTORCH_EXTENSION_NAME=_kfamd_ops",
                                                  "-DHIP_ENABLE_WARP_SYNC_BUILTINS=1"]
    link = ["-shared", "-fPIC", f"--offload-arch={ARCH}", f"-L{lib}", f"-Wl,-rpath,{lib}",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lamdhip64"]
    return kernel, binding, link


# per-source extra flags: flash_attn.hip's kernels were tuned (and their code is pinned,
# tests/test_kernels_static.py) with the MFMA accumulators in the VGPR form, and are built
# without SLP vectorization: it packed the softmax's f32 adds / multiplies into v_pk_*_f32,
# which cost more issue slots beside the MFMAs than the scalar ops (attention backward 7.50 ->
# 7.26 ms at B4 S8192, profiles/fa_fwd128_r5.md)
FILE_FLAGS = {"flash_attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"]}


def _sources():
    hips = sorted(CSRC.glob("*.hip"))
    return hips, CSRC / "bindings.cpp"


def _digest(files, flags) -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    for hdr in sorted(CSRC.glob("*.h")):
        h.update(hdr.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _run(cmd):
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
    return p.stderr


def _toolchain_key() -> list[str]:
    """Everything the compile and link flags are derived from, WITHOUT importing
    ``torch.utils.cpp_extension`` (0.2-0.3 s per worker process): the flags come from torch's
    install directory, version and C++ ABI, the ROCm root and this module's own constants, so
    hashing those identifies them.  ``_flags()`` runs only when a rebuild is needed."""
    import torch

    return [ARCH, HIPCC, torch.__version__, os.path.dirname(torch.__file__),
            str(int(torch._C._GLIBCXX_USE_CXX11_ABI)), os.environ.get("ROCM_HOME", "/opt/rocm"),
            hashlib.sha256(Path(__file__).read_bytes()).hexdigest()[:16],
            *(f"{k}:{v}" for k, v in sorted(FILE_FLAGS.items()))]


def current_digest() -> str:
    hips, bind = _sources()
    return _digest(hips + [bind], _toolchain_key())


def up_to_date() -> bool:
    """True when the in-tree library was built from exactly these sources and toolchain."""
    stamp = HERE / (LIB_NAME + ".stamp")
    return LIB_PATH.exists() and stamp.exists() and stamp.read_text().strip() == current_digest()


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    hips, bind = _sources()
    digest = current_digest()
    stamp = HERE / (LIB_NAME + ".stamp")
    if not force and LIB_PATH.exists() and stamp.exists() and stamp.read_text().strip() == digest:
        return LIB_PATH
    # several ranks of one node may find the library stale together: one builds, the others
    # wait on the lock and then see the fresh stamp
    import fcntl
    with open(HERE / (LIB_NAME + ".lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and LIB_PATH.exists() and stamp.exists() and stamp.read_text().strip() == digest:
            return LIB_PATH
        return _build_locked(hips, bind, digest, stamp, jobs, verbose)


def _build_locked(hips, bind, digest, stamp, jobs, verbose) -> Path:
    kernel, binding, link = _flags()
    BUILD.mkdir(exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    cmds, objs = [], []
    for src in hips:
        obj = BUILD / (src.stem + ".o")
        objs.append(obj)
        cmds.append([HIPCC, *kernel, *FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)])
    bobj = BUILD / "bindings.o"
    objs.append(bobj)
    cmds.append([HIPCC, *binding, "-x", "c++", "-c", str(bind), "-o", str(bobj)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for err in ex.map(_run, cmds):
            if verbose and err:
                print(err, file=sys.stderr)
    tmp = HERE / (LIB_NAME + ".tmp")
    _run([HIPCC, *link, *map(str, objs), "-o", str(tmp)])
    os.replace(tmp, LIB_PATH)
    stamp.write_text(digest)
    return LIB_PATH


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    p = build(force=a.force, jobs=a.j, verbose=a.v)
    print(p)


if __name__ == "__main__":
    main()
