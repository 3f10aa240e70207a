#!/bin/bash
# Round 4b: persistent NT GEMM ablation (full / no DMA / MFMA only) vs hipBLASLt,
# interleaved timing + PMC passes on the fc2-forward shape.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u scripts/gemm_ablation.py 2>&1 | tee gpurun_out/r4b_gemm_ablation.txt || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for S in "16384 4096 11008" "16384 4096 4096"; do
  tag=$(echo $S | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA --kernel-trace --output-format csv -d gpurun_out/r4b_p1_$tag -o w -- python3 scripts/gemm_ablation_once.py $S > gpurun_out/r4b_p1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/r4b_p2_$tag -o w -- python3 scripts/gemm_ablation_once.py $S > gpurun_out/r4b_p2_$tag.log 2>&1 || exit 1
  echo "== $S"
  python3 scripts/summarize_ablation_pmc.py gpurun_out/r4b_p1_$tag gpurun_out/r4b_p2_$tag | tee -a gpurun_out/r4b_pmc.txt
done
