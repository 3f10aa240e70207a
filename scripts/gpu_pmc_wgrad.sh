#!/bin/bash
# PMC counters for the wgrad kernel (no sys/runtime trace, per the pool rules).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc1 -o w -- python3 scripts/wgrad_once.py > gpurun_out/pmc1.log 2>&1
echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc2 -o w -- python3 scripts/wgrad_once.py > gpurun_out/pmc2.log 2>&1
echo "pmc2 rc=$?"
