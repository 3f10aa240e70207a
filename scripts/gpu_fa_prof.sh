#!/bin/bash
# Per-kernel FA timing (stats) for two backward occupancy variants + PMC counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for occ in ${OCCS:-11 22}; do
  EMA_FA_BWD_OCC=$occ timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/faprof_$occ -o f --output-format csv -- python3 scripts/fa_bench.py > gpurun_out/faprof_$occ.log 2>&1 || { echo prof failed; tail -20 gpurun_out/faprof_$occ.log; exit 1; }
  f=$(find gpurun_out/faprof_$occ -name "*kernel_stats.csv" | head -1)
  echo "== occ $occ"; cut -d, -f1-5 "$f" | cut -c1-150 | head -8
done
EMA_FA_BWD_OCC=${PMC_OCC:-22} timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY --kernel-trace --output-format csv -d gpurun_out/fapmc -o f -- python3 scripts/fa_bench.py > gpurun_out/fapmc.log 2>&1 || { echo pmc failed; tail -20 gpurun_out/fapmc.log; exit 1; }
echo pmc ok
