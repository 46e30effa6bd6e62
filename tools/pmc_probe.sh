#!/bin/bash
# SQ-counter probe of the NTT pass and MSM accumulation kernels (two --pmc passes each, one
# program run per pass).  Usage on the GPU box: bash tools/pmc_probe.sh <tag>
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=${1:-probe}
mkdir -p gpurun_out/$T
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for p in A B; do
  timeout -s KILL 150 rocprofv3 --pmc ${!p} --kernel-include-regex 'k_ntt_pass|k_accum_level0|k_bucket_reduce' --output-format csv -d gpurun_out/$T/ntt_$p -o run -- python3 tools/ntt_bench.py --log 26 --reps 1 > gpurun_out/$T/ntt_$p.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc ${!p} --kernel-include-regex 'k_ntt_pass|k_accum_level0|k_bucket_reduce' --output-format csv -d gpurun_out/$T/msm_$p -o run -- python3 tools/msm_bench.py --log-rows 24 --reps 1 > gpurun_out/$T/msm_$p.log 2>&1
done
echo probe done
