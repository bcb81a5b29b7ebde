#!/bin/bash
# Separate rocprofv3 --pmc passes for one kernel of a bench command (MI355X_MICROARCH.md: TCC has
# 4 slots, FETCH_SIZE costs 3 and WRITE_SIZE 2, so they get their own passes; SQ has 8).
# usage: tools/prof_passes.sh OUTDIR KERNEL_REGEX -- cmd args...
set -o pipefail
out=$1; kre=$2; shift 3
mkdir -p "$out"
passes=(
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS"
  "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"
  "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"
)
# MFMA busy (k_hex_mfma configs): PASS_MFMA=1 adds the pass
[ "${PASS_MFMA:-0}" = 1 ] && passes+=("SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE")
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 300 rocprofv3 --kernel-include-regex "$kre" --pmc $p -d "$out/pass$i" -o run --output-format csv -- "$@" > "$out/pass$i.log" 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
  i=$((i+1))
done
echo "passes ok"
