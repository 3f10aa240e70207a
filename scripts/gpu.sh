#!/bin/bash
# One parametrised GPU runner for gpurun (replaces the per-experiment
# scripts/gpu_r*.sh launchers):
#
#   bash scripts/gpu.sh TAG STEP [STEP ...]
#
# Every step runs under its own time limit, logs to gpurun_out/TAG_STEP.log,
# and the first failing step ends the call (no GPU work after a fault, an
# abort or a time limit).  Steps:
#   tests      pytest -m gpu (one process)
#   quick      pytest -m gpu on the kernel / GEMM numerics files only
#   pyt        pytest -m gpu $PYTEST_ARGS (a chosen subset)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py --steps 8 --warmup 2 (the headline config)
#   prof       rocprofv3 --kernel-trace --stats over bench.py --steps 2 --warmup 1
#   prof4k / bench4k  the same profile / bench at seq 4096, micro-batch 4
#   profpx7    rocprofv3 kernel trace of the llama7b-tp8 proxy (profpx70: llama70b-tp8)
#   ab         bench.py twice plain / twice with $AB_ENV, interleaved
#   scriptab   python $SCRIPT plain / with $AB_ENV, interleaved twice
#   ltre       scripts/lt_retune.py (torch.matmul's hipBLASLt pick vs the best solution)
#   lab        scripts/gemm_lab.py (bench-only GEMM builds vs production vs hipBLASLt)
#   gemm       scripts/gemm_nt_bench.py (in-model NT shapes vs hipBLASLt)
#   wgrad      scripts/wgrad_ab.py (4-wave vs 8-wave wgrad vs hipBLASLt)
#   px7ab      the TP8 proxy plain, then with $AB_ENV
#   fa         scripts/fa_bench.py
#   faab       scripts/fa_bench.py plain / with $AB_ENV, interleaved twice
#   px7        bench.py --proxy llama7b-tp8 (one TP rank, simulated TP)
#   px70       bench.py --proxy llama70b-tp8
#   pmc_lab    rocprofv3 --pmc passes over scripts/gemm_lab.py (one pass per run)
#   pmc_gemms  one rocprofv3 --pmc pass over the NT GEMM bench and the wgrad A/B
# Extra bench.py arguments: BENCH_ARGS="..." in the environment.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1
shift
[ -n "$TAG" ] || { echo "usage: gpu.sh TAG STEP..."; exit 2; }

run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  local log="gpurun_out/${TAG}_${name}.log"
  echo "== ${name} (limit ${secs}s)"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  tail -n 4 "$log" | cut -c1-600
  if [ $rc -ne 0 ]; then
    echo "step ${name} failed rc=${rc}"
    tail -n 40 "$log"
    exit 1
  fi
}

prof() {  # prof NAME SECONDS CMD...  (rocprofv3 kernel trace + stats)
  local name=$1 secs=$2
  shift 2
  export TMPDIR=/tmp
  run "$name" "$secs" rocprofv3 --kernel-trace --stats --output-format csv \
    -d "gpurun_out/${TAG}_${name}" -o prof -- "$@"
  find "gpurun_out/${TAG}_${name}" -name "*kernel_stats.csv" | head -3
}

for step in "$@"; do
  case $step in
    tests) run tests 1000 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
             -p no:cacheprovider tests -m gpu ;;
    quick) run quick 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
             -p no:cacheprovider tests/test_kernels_gpu.py tests/test_gemm_gpu.py -m gpu ;;
    pyt) run pyt 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
             -p no:cacheprovider -m gpu $PYTEST_ARGS ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 500 python -u bench.py --steps 8 --warmup 2 $BENCH_ARGS ;;
    prof) prof prof 600 python3 -u bench.py --steps 2 --warmup 1 $BENCH_ARGS ;;
    prof4k) prof prof4k 600 python3 -u bench.py --seq_len 4096 --micro_batch 4 --steps 2 --warmup 1 ;;
    bench4k) run bench4k 500 python -u bench.py --seq_len 4096 --micro_batch 4 --steps 6 --warmup 2 ;;
    profpx7) prof profpx7 600 python3 -u bench.py --proxy llama7b-tp8 --steps 2 --warmup 1 ;;
    profpx70) prof profpx70 900 python3 -u bench.py --proxy llama70b-tp8 --steps 1 --warmup 1 ;;
    ab)  # interleaved bench A/B: plain, then with $AB_ENV (e.g. AB_ENV="EMA_X=1"), twice
      for i in 1 2; do
        run "ab${i}a" 400 python -u bench.py --steps 6 --warmup 2 $BENCH_ARGS
        run "ab${i}b" 400 env $AB_ENV python -u bench.py --steps 6 --warmup 2 $BENCH_ARGS
      done
      for f in gpurun_out/${TAG}_ab*.log; do
        echo "$f $(grep -o '"value": [0-9.]*' "$f")"
      done ;;
    ltre) run ltre 500 python -u scripts/lt_retune.py ;;
    scriptab)  # $SCRIPT plain, then with $AB_ENV, interleaved twice
      for i in 1 2; do
        run "sab${i}a" 300 python -u $SCRIPT
        run "sab${i}b" 300 env $AB_ENV python -u $SCRIPT
      done
      tail -n 5 gpurun_out/${TAG}_sab?[ab].log ;;
    lab) run lab 400 python -u scripts/gemm_lab.py $LAB_SHAPES ;;
    gemm) run gemm 400 python -u scripts/gemm_nt_bench.py --variants ${NT_VARIANTS:-5,6} ;;
    wgrad) run wgrad 400 python -u scripts/wgrad_ab.py ;;
    px70ab)  # 70B TP8 proxy, plain then with $AB_ENV
      run px70a 700 python -u bench.py --proxy llama70b-tp8 --steps 3 --warmup 1
      run px70b 700 env $AB_ENV python -u bench.py --proxy llama70b-tp8 --steps 3 --warmup 1 ;;
    px7ab)  # TP8 proxy, plain then with $AB_ENV
      run px7a 500 python -u bench.py --proxy llama7b-tp8 --steps 6 --warmup 2
      run px7b 500 env $AB_ENV python -u bench.py --proxy llama7b-tp8 --steps 6 --warmup 2 ;;
    fa) run fa 400 python -u scripts/fa_bench.py ;;
    faab)  # FA timing plain, then with $AB_ENV, twice
      for i in 1 2; do
        run "fa${i}a" 300 python -u scripts/fa_bench.py
        run "fa${i}b" 300 env $AB_ENV python -u scripts/fa_bench.py
      done
      grep -h "fwd" gpurun_out/${TAG}_fa?[ab].log ;;
    px7) run px7 500 python -u bench.py --proxy llama7b-tp8 --steps 6 --warmup 2 ;;
    px70) run px70 700 python -u bench.py --proxy llama70b-tp8 --steps 3 --warmup 1 ;;
    pmc_fa)  # FA forward counters, plain then with $AB_ENV (one pass per run)
      export TMPDIR=/tmp
      i=0
      for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
                 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        run "pmcfa${i}a" 60 rocprofv3 --pmc $ctr --output-format csv -d "gpurun_out/${TAG}_pmcfa_a${i}" -o pmc -- \
          python3 -u scripts/fa_pmc_one.py
        export $AB_ENV
        run "pmcfa${i}b" 60 rocprofv3 --pmc $ctr --output-format csv -d "gpurun_out/${TAG}_pmcfa_b${i}" -o pmc -- \
          python3 -u scripts/fa_pmc_one.py
        unset ${AB_ENV%%=*}
      done
      python scripts/pmc_table.py gpurun_out/${TAG}_pmcfa_a* > "gpurun_out/${TAG}_pmcfa_a.txt" 2>&1
      python scripts/pmc_table.py gpurun_out/${TAG}_pmcfa_b* > "gpurun_out/${TAG}_pmcfa_b.txt" 2>&1
      grep -A2 "fa_fwd" "gpurun_out/${TAG}_pmcfa_a.txt" "gpurun_out/${TAG}_pmcfa_b.txt" | cut -c1-600 ;;
    pmc_gemms)  # one PMC pass over the NT GEMM bench (variant 6) and the wgrad A/B
      export TMPDIR=/tmp
      CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
      run pmcnt 120 rocprofv3 --pmc $CTR --output-format csv -d "gpurun_out/${TAG}_pmcnt" -o pmc -- \
        python3 -u scripts/gemm_nt_bench.py --variants 6 --rounds 1 --iters 2
      run pmcwg 120 rocprofv3 --pmc $CTR --output-format csv -d "gpurun_out/${TAG}_pmcwg" -o pmc -- \
        python3 -u scripts/wgrad_ab.py
      python scripts/pmc_table.py gpurun_out/${TAG}_pmcnt > "gpurun_out/${TAG}_pmcnt_table.txt" 2>&1
      python scripts/pmc_table.py gpurun_out/${TAG}_pmcwg > "gpurun_out/${TAG}_pmcwg_table.txt" 2>&1
      grep -h -A2 "wgrad\|gemm_nt6\|Cijk" gpurun_out/${TAG}_pmcnt_table.txt gpurun_out/${TAG}_pmcwg_table.txt | cut -c1-300 ;;
    pmc_lab)
      export TMPDIR=/tmp
      i=0
      for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
                 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
                 "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
                 "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        run "pmc${i}" 120 rocprofv3 --pmc $ctr --output-format csv -d "gpurun_out/${TAG}_pmc${i}" -o pmc -- \
          python3 -u scripts/gemm_lab.py $LAB_SHAPES
      done
      python scripts/pmc_table.py gpurun_out/${TAG}_pmc* > "gpurun_out/${TAG}_pmc_table.txt" 2>&1
      cat "gpurun_out/${TAG}_pmc_table.txt" | cut -c1-400 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
