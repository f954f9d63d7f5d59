#!/bin/bash
# One parameterised GPU session (the only gpurun script; recipes in tools/RECIPES.md):
#
#   tools/gpu_session.sh OUTDIR STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failure (non-zero status, a
# time limit, an abort or a fault) ends the session, so nothing more touches the GPU after it.
#   tests[:K_EXPR]          pytest -m gpu (optionally -k K_EXPR)              -> OUTDIR/pytest.log
#   smoke                   __graft_entry__.smoke()                             -> OUTDIR/smoke.log
#   bench[:STEPS[:WARMUP]]  python bench.py (+ $BENCH_ARGS)                     -> OUTDIR/bench*.log
#   prof[:STEPS]            rocprofv3 --kernel-trace --stats of bench.py (STEPS + 2 warm-up steps traced), per-step summary
#                                                                               -> OUTDIR/prof/summary.md
#   proftool:SCRIPT[:A,..]  rocprofv3 --kernel-trace --stats of python3 tools/SCRIPT A ..
#                                                                               -> OUTDIR/proftool_N/kernel_stats.csv
#   pmctool:SCRIPT[:A,..]   the two PMC passes of tools/kbench/pmc.sh over python3 tools/SCRIPT A ..
#                                                                               -> OUTDIR/pmctool_N/
#   kbench:BIN[:A,B,..]     tools/kbench/bin/BIN A B ..                         -> OUTDIR/kbench.txt
#                           (exit 3 = the bench's numerics check failed: recorded, not fatal)
#   pmc:BIN[:A,B,..]        two PMC passes over a kbench binary (tools/kbench/pmc.sh)
#   tool:SCRIPT[:A,B,..]    python -u tools/SCRIPT A B ..                       -> OUTDIR/SCRIPT.log
#   env:VAR=VALUE           export VAR=VALUE for the steps after it (env:VAR= unsets it)
#   ext:FILE                install the prebuilt extension FILE as ops/_kfamd_ops.so for the steps
#                           after it (A/B of two builds in one session; the tree's own build is put
#                           back when the session ends)
# Counter runs never combine --pmc with trace domains; nothing here sets GPU_MAX_HW_QUEUES.
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=${1:?usage: gpu_session.sh OUTDIR STEP...}
shift
mkdir -p "$O"
n=0
EXT=service_account_auth_improvements_amd/ops/_kfamd_ops.so
EXT_SAVED=""
restore_ext() { [ -n "$EXT_SAVED" ] && cp "$EXT_SAVED" "$EXT"; }
trap restore_ext EXIT

fail() { echo "step '$1' failed rc=$2"; [ -f "$3" ] && tail -40 "$3"; exit "$2"; }

for step in "$@"; do
  n=$((n + 1))
  IFS=: read -r kind a1 a2 <<< "$step"
  args=()
  [ -n "$a2" ] && IFS=, read -r -a args <<< "$a2"
  echo "=== [$n] $step ($(date +%T))"
  case "$kind" in
    tests)
      log=$O/pytest.log
      [ -f "$log" ] && log=$O/pytest_$n.log     # a second tests step in one session keeps the first log
      k=(); [ -n "$a1" ] && k=(-k "$a1")
      timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests "${k[@]}" > "$log" 2>&1 \
        || fail "$step" $? "$log"
      tail -1 "$log" ;;
    smoke)
      log=$O/smoke.log
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail "$step" $? "$log"
      tail -1 "$log" ;;
    bench)
      log=$O/bench_$n.log
      timeout -k 10 700 python -u bench.py --steps "${a1:-20}" --warmup "${a2:-5}" $BENCH_ARGS > "$log" 2>&1 \
        || fail "$step" $? "$log"
      tail -1 "$log" | cut -c1-400 ;;
    prof)
      log=$O/prof.log
      timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 bench.py --steps "${a1:-3}" --warmup 2 --crd-jobs 0 $BENCH_ARGS > "$log" 2>&1 || fail "$step" $? "$log"
      f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
      python tools/prof_summary.py "$f" "$(( ${a1:-3} + 2 ))" > "$O/prof/summary.md" && cp "$f" "$O/prof/kernel_stats.csv"
      head -18 "$O/prof/summary.md" ;;
    proftool)
      d=$O/proftool_$n
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- \
        python3 "tools/$a1" "${args[@]}" > "$d.log" 2>&1 || fail "$step" $? "$d.log"
      f=$(find "$d" -name "*kernel_stats.csv" | head -1)
      cp "$f" "$d/kernel_stats.csv" && head -25 "$d/kernel_stats.csv" | cut -c1-200 ;;
    pmctool)
      # the two counter passes of tools/kbench/pmc.sh over python3 tools/SCRIPT (no trace domains)
      d=$O/pmctool_$n
      mkdir -p "$d"
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU --output-format csv -d "$d" -o p1 -- \
        python3 "tools/$a1" "${args[@]}" > "$d/p1.log" 2>&1 || fail "$step" $? "$d/p1.log"
      timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY \
        --output-format csv -d "$d" -o p2 -- python3 "tools/$a1" "${args[@]}" > "$d/p2.log" 2>&1 || fail "$step" $? "$d/p2.log"
      find "$d" -name "*counter_collection.csv" ;;
    kbench)
      log=$O/kbench.txt
      echo "=== $a1 ${args[*]}" >> "$log"
      # rc 3 is the benches' own "numerics mismatch" exit (the kernel ran to completion and
      # the GPU is fine): recorded, and the session goes on
      rc=0; timeout -k 5 120 "tools/kbench/bin/$a1" "${args[@]}" >> "$log" 2>&1 || rc=$?
      if [ $rc -eq 3 ]; then echo "numerics mismatch (rc 3) recorded in $log"
      elif [ $rc -ne 0 ]; then fail "$step" $rc "$log"; fi
      sed -n '/=== '"$a1"'/,$p' "$log" | tail -12 ;;
    pmc)
      bash tools/kbench/pmc.sh "$O/pmc_$n" "$a1" "${args[@]}" || fail "$step" $? ""
      ;;
    tool)
      log=$O/${a1%.py}_$n.log
      timeout -k 10 600 python -u "tools/$a1" "${args[@]}" > "$log" 2>&1 || fail "$step" $? "$log"
      grep -v amdgpu.ids "$log" | tail -8 | cut -c1-300 ;;
    ext)
      [ -f "$a1" ] || { echo "ext: no file $a1"; exit 2; }
      if [ -z "$EXT_SAVED" ]; then EXT_SAVED=$O/.ext_saved.so; cp "$EXT" "$EXT_SAVED"; fi
      cp "$a1" "$EXT"
      echo "ext $a1" ;;
    env)
      v=${step#env:}
      if [ -z "${v#*=}" ]; then unset "${v%%=*}"; else export "$v"; fi
      echo "env $v" ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
done
echo "=== session done ($n steps)"
