"""Per-step kernel timeline analysis of a rocprofv3 kernel trace: finds the decode steps (by
the LM-head GEMM marker or a name substring), and reports busy vs wall time and the top
kernels inside the window of the last N steps."""
import csv, re, sys, collections
path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "decode_combine"
per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 32
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
# last 8 steps worth of marker hits
take = idx[-8 * per_step:]
lo, hi = take[0], take[-1]
win = rows[lo:hi + 1]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(win, win[1:])]
print(f"window {len(win)} kernels, wall {(t1-t0)/1e3:.1f} us, busy {busy/1e3:.1f} us ({100*busy/(t1-t0):.0f}%), "
      f"mean gap {sum(gaps)/len(gaps)/1e3:.2f} us, kernels/step {len(win)/8:.0f}")
agg = collections.defaultdict(lambda: [0, 0])
for r in win:
    n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""))[:70]
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:15]:
    print(f"{n:72s} {c/8:6.0f}/step {t/c/1e3:8.2f} us avg {t/8/1e3:9.1f} us/step")
