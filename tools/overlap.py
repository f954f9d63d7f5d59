"""How much of kernel family A's time ran concurrently with other kernels (rocprofv3 trace)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), pat in r["Kernel_Name"]) for r in rows]
A = sorted((s, e) for s, e, a in iv if a)
B = sorted((s, e) for s, e, a in iv if not a)
tot = sum(e - s for s, e in A)
ov = 0
j = 0
for s, e in A:
    for bs, be in B:
        if be <= s or bs >= e:
            continue
        ov += min(e, be) - max(s, bs)
print(f"{pat}: {len(A)} kernels, {tot/1e6:.2f} ms total, {ov/1e6:.2f} ms overlapped with other kernels "
      f"({100*ov/max(tot,1):.0f}%)")
