"""Summarise a rocprofv3 kernel_stats.csv: top kernels, grouped categories, per-step time."""
import csv, sys, re
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
cats = {}
def cat(n):
    if n.startswith('Cijk') or 'Custom_Cijk' in n: return 'GEMM (hipBLASLt)'
    if 'gemm_tn' in n: return 'GEMM dW (HIP, MFMA 16x16x32)'
    if 'flash_fwd' in n: return 'attention fwd (HIP)'
    if 'flash_bwd' in n: return 'attention bwd (HIP)'
    if 'adamw' in n or 'sumsq' in n or 'sum_final' in n: return 'optimizer (HIP)'
    if 'rmsnorm' in n or 'colsum' in n: return 'rmsnorm (HIP)'
    if 'swiglu' in n: return 'swiglu (HIP)'
    if 'rope' in n: return 'rope (HIP)'
    if 'transpose_bf16' in n: return 'weight transpose for dX (HIP)'
    if 'embed_' in n: return 'embedding (HIP)'
    if 'ce_kernel' in n: return 'cross-entropy (HIP)'
    if 'attn_fwd' in n or 'bwd_kernel' in n or 'bwd_preprocess' in n: return 'attention (SDPA/AOTriton)'
    return 'other (torch/runtime)'
for r in rows:
    c = cat(r['Name']); cats[c] = cats.get(c, 0) + float(r['TotalDurationNs'])
print(f"total kernel time {tot/1e6:.1f} ms over {steps:g} steps = {tot/1e6/steps:.1f} ms/step")
print("| category | ms/step | % |\n|---|---|---|")
for c, v in sorted(cats.items(), key=lambda x: -x[1]):
    print(f"| {c} | {v/1e6/steps:.2f} | {100*v/tot:.1f} |")
print("\n| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:20]:
    n = re.sub(r'\(.*', '', r['Name'])[:90]
    print(f"| {n} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
