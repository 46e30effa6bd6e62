#!/bin/bash
# SQ counters of the NTT pass kernel (two --pmc passes, one program run each): where a pass's wave cycles
# go (VALU issue, waits on memory / barriers, LDS).  Usage on the GPU box: bash tools/pmc_ntt.sh <tag>
cd "$GRAFT_REPO_ROOT" || exit 1; export TMPDIR=/tmp
T=${1:-ntt}
mkdir -p gpurun_out/$T
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM"
for p in A B; do
  timeout -s KILL 150 rocprofv3 --pmc ${!p} --kernel-include-regex 'k_ntt_pass' --output-format csv -d gpurun_out/$T/ntt_$p -o run -- python3 tools/ntt_bench.py --log 26 --reps 1 > gpurun_out/$T/ntt_$p.log 2>&1 || { echo "pass $p failed"; exit 1; }
done
echo probe done
