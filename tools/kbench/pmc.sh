#!/bin/bash
# PMC passes over a microbench binary: pmc.sh OUTDIR BIN [args]; one counter group per run.
set -o pipefail
export TMPDIR=/tmp
out=$1; b=$2; shift 2
mkdir -p $out
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_SALU --output-format csv -d $out -o p1 -- tools/kbench/bin/$b "$@" > $out/p1.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY --output-format csv -d $out -o p2 -- tools/kbench/bin/$b "$@" > $out/p2.log 2>&1 || exit $?
find $out -name "*counter_collection.csv"
