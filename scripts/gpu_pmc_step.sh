#!/bin/bash
# PMC counters over one Llama-2-7B training step (bench.py), one pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 420 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_$name -o p \
    -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmc_$name.log 2>&1 || { echo "pmc $name failed rc=$?"; tail -5 gpurun_out/pmc_$name.log; return 1; }
  echo "pmc $name ok"
}
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE &&
run fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
run write WRITE_SIZE &&
python scripts/summarize_pmc.py gpurun_out/pmc_summary.csv gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write &&
head -30 gpurun_out/pmc_summary.csv | cut -c1-200
