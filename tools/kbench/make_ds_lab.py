"""Regenerate tools/kbench/decode_step_lab.hip from ops/csrc/decode_step.hip with ablation knobs:
KF_DS_NOBAR=1 (drain, no barrier poll) / 2 (no barrier), KF_DS_NOATT=1 (no attention phase),
KF_DS_NODMA=1 (no weight DMA).  The shipped kernel carries none of them."""
import os

here = os.path.dirname(os.path.abspath(__file__))
src = os.path.join(here, "../../service_account_auth_improvements_amd/ops/csrc/decode_step.hip")
s = open(src).read()
s = s.replace('#include "common.h"', "// LAB COPY of ops/csrc/decode_step.hip with ablation knobs (tools/kbench/make_ds_lab.py); "
              "never shipped.\n#include \"common.h\"\n#ifndef KF_DS_NOBAR\n#define KF_DS_NOBAR 0\n#endif\n"
              "#ifndef KF_DS_NOATT\n#define KF_DS_NOATT 0\n#endif\n#ifndef KF_DS_NODMA\n#define KF_DS_NODMA 0\n#endif", 1)
old = ("  auto grid_barrier = [&](int k) -> bool {\n"
       "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");          // every wave drains its stores\n"
       "    __syncthreads();")
assert old in s
s = s.replace(old, "  auto grid_barrier = [&](int k) -> bool {\n#if KF_DS_NOBAR == 2\n    __syncthreads();\n    return true;\n#endif\n"
              "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n    __syncthreads();\n#if KF_DS_NOBAR == 1\n"
              "    return true;\n#endif")
old = "    if (g < M * HKV * ns) {"
assert old in s
s = s.replace(old, "    if (!KF_DS_NOATT && g < M * HKV * ns) {")
old = "__device__ __forceinline__ void dma_piece(const char* src, u32 lds, u32 voff) {\n"
assert old in s
s = s.replace(old, old + "  if (KF_DS_NODMA) return;\n")
for m in (1, 2, 3, 4):   # KF_DS_RS<m> / KF_DS_PF<m> override the tuned ring / prefetch constants
    import re
    s = re.sub(r"template <> struct Cfg<%d> { static constexpr int RS = (\d+), PF = (\d+); };" % m,
               lambda mo: ("#ifndef KF_DS_RS%d\n#define KF_DS_RS%d %s\n#endif\n#ifndef KF_DS_PF%d\n#define KF_DS_PF%d %s\n#endif\n"
                           "template <> struct Cfg<%d> { static constexpr int RS = KF_DS_RS%d, PF = KF_DS_PF%d; };")
               % (m, m, mo.group(1), m, m, mo.group(2), m, m, m), s)
s = s.replace('extern "C" ', 'extern "C" __attribute__((weak)) ')
open(os.path.join(here, "decode_step_lab.hip"), "w").write(s)
