#!/bin/bash
# Round 4aa: FA PMC after the round-4 VALU cuts (Llama-2-7B s=1k shape), one rocprofv3 pass per counter set.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
SH=16,1024,32,32,128
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcfa_t -o f -- python3 scripts/fa_bench2.py $SH > gpurun_out/pmcfa_t.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcfa_1 -o f -- python3 scripts/fa_bench2.py $SH > gpurun_out/pmcfa_1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmcfa_2 -o f -- python3 scripts/fa_bench2.py $SH > gpurun_out/pmcfa_2.log 2>&1 && \
python3 scripts/summarize_fa_pmc.py gpurun_out/pmcfa_t gpurun_out/pmcfa_1 gpurun_out/pmcfa_2 > gpurun_out/r4aa_pmc_fa.txt && cat gpurun_out/r4aa_pmc_fa.txt
