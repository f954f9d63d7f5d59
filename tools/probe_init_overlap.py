"""CRD-to-first-step probe: can a worker overlap HIP runtime / device initialisation with the
torch import?  Each variant runs in fresh processes (several times, alternating):

  serial  : import torch; torch.cuda.set_device(0); first allocation
  overlap : a thread runs hipInit / hipSetDevice / hipFree(0) through ctypes while the main
            thread imports torch; then the same torch calls

Prints one JSON line per run with the time from process start to "device ready" and the
import time; a summary line with the medians."""
import json
import os
import statistics
import subprocess
import sys

CHILD = r'''
import os, sys, time, json, threading
t0 = time.perf_counter()
mode = sys.argv[1]
th = None
if mode == "overlap":
    def hip_init():
        import ctypes
        lib = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        lib.hipInit(0)
        lib.hipSetDevice(0)
        lib.hipFree(None)
    th = threading.Thread(target=hip_init, daemon=True)
    th.start()
import torch
t_imp = time.perf_counter() - t0
if th is not None:
    th.join()
t_join = time.perf_counter() - t0
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
print(json.dumps({"mode": mode, "import_s": round(t_imp, 3), "joined_s": round(t_join, 3),
                  "device_ready_s": round(time.perf_counter() - t0, 3)}))
'''


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    res = {"serial": [], "overlap": []}
    for _ in range(reps):
        for mode in ("serial", "overlap"):
            out = subprocess.run([sys.executable, "-c", CHILD, mode], capture_output=True, text=True, timeout=120)
            line = [x for x in out.stdout.splitlines() if x.startswith("{")]
            if not line:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(1)
            rec = json.loads(line[-1])
            print(json.dumps(rec), flush=True)
            res[mode].append(rec["device_ready_s"])
    print(json.dumps({"median_device_ready_s": {m: statistics.median(v) for m, v in res.items()}}))


if __name__ == "__main__":
    main()
