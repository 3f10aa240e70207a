#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python scripts/fa_bench.py > gpurun_out/fa_bench.log 2>&1; echo "bench rc=$?"; cat gpurun_out/fa_bench.log | grep iter
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmcfa1 -o f -- python3 scripts/fa_bench.py > gpurun_out/pmcfa1.log 2>&1
echo "pmc1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmcfa2 -o f -- python3 scripts/fa_bench.py > gpurun_out/pmcfa2.log 2>&1
echo "pmc2 rc=$?"
