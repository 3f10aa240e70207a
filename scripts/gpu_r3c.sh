#!/bin/bash
# Round 3: 7B step with the fused GLU MLP (hipBLASLt plain GEMMs) vs unfused,
# SP piece-GEMM overhead, simulated-TP proxies, NT GEMM PMC on the fc2 shape.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u scripts/fa_diag.py --json gpurun_out/r3c_fa_diag.json > gpurun_out/r3c_fa_diag.txt 2>&1 || { tail -20 gpurun_out/r3c_fa_diag.txt; exit 1; }
cat gpurun_out/r3c_fa_diag.txt
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3c_bench_fused.log 2>&1 || { tail -20 gpurun_out/r3c_bench_fused.log; exit 1; }
tail -1 gpurun_out/r3c_bench_fused.log
EMA_FUSED_MLP=0 timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3c_bench_unfused.log 2>&1 || { tail -20 gpurun_out/r3c_bench_unfused.log; exit 1; }
tail -1 gpurun_out/r3c_bench_unfused.log
timeout -k 10 200 python -u scripts/sp_overlap_bench.py --json gpurun_out/r3c_sp_pieces.json > gpurun_out/r3c_sp_pieces.txt 2>&1 || { tail -20 gpurun_out/r3c_sp_pieces.txt; exit 1; }
cat gpurun_out/r3c_sp_pieces.txt
timeout -k 10 400 python -u bench.py --proxy llama7b-tp8 --steps 4 --warmup 2 > gpurun_out/r3c_px_l7tp8.log 2>&1 || { tail -20 gpurun_out/r3c_px_l7tp8.log; exit 1; }
tail -1 gpurun_out/r3c_px_l7tp8.log
timeout -k 10 500 python -u bench.py --proxy llama70b-tp8 --steps 3 --warmup 1 > gpurun_out/r3c_px_l70tp8.log 2>&1 || { tail -20 gpurun_out/r3c_px_l70tp8.log; exit 1; }
tail -1 gpurun_out/r3c_px_l70tp8.log
bash scripts/gpu_r3b.sh > gpurun_out/r3c_pmc.txt 2>&1 || { tail -20 gpurun_out/r3c_pmc.txt; exit 1; }
cat gpurun_out/r3c_pmc.txt
