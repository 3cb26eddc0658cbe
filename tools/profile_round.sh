#!/bin/bash
# Round profile: kernel trace + stats over bench.py, then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE) on the bulge chase and the two streaming
# band-reduction kernels (X/M and the rank-64 update) at n = 4096, the same
# two passes over one n = 12,288 solve (band update, X/M and the pivot
# order's Schur updates: HBM-resident there), then the per-class traffic
# JSONs (X/M with its algorithmic bytes), one MFMA-busy pass over the MFMA
# kernels (tools/mfma_busy.py), the stall passes over X/M, the band update
# and the Schur update at n = 12,288 (tools/stall_passes.py picks the
# counters the box lists; tools/stall_summary.py), then the default bench
# line.  Every GPU step has its own limit and the steps are chained, so the
# first failure ends the script.
# usage: tools/profile_round.sh OUTDIR
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/${1:-gpurun_out/prof}
KRE="bulge_df_kernel|bulge_lds_kernel|syr2k_w|xm_kernel"
LRE="syr2k_w|xm_kernel|syrk_compact"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-large-n --no-e2e > "$OUT/trace_bench.log" 2>&1
echo "trace done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -f csv -d "$OUT/pmc_$C" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-syrk --no-large-n --no-e2e > "$OUT/pmc_$C.log" 2>&1
  echo "pmc $C done"
done
N=12288 ROWS=2 REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace12k" -o run -- \
  python3 tools/solve_time.py > "$OUT/trace12k.log" 2>&1
for C in FETCH_SIZE WRITE_SIZE; do
  N=12288 ROWS=2 REPS=1 timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$LRE" -f csv -d "$OUT/pmc12k_$C" -o run -- \
    python3 tools/solve_time.py > "$OUT/pmc12k_$C.log" 2>&1
  echo "pmc12k $C done"
done
first() { find "$1" -name "$2" | sort | sed -n 1p; }
python3 tools/pmc_traffic.py "$OUT/pmc_traffic.json" "$(first $OUT/pmc_FETCH_SIZE '*counter_collection.csv')" \
  "$(first $OUT/pmc_WRITE_SIZE '*counter_collection.csv')" "$(first $OUT/trace '*kernel_stats.csv')" \
  bulge_chase=bulge_df_kernel band_update=syr2k_w band_xm=xm_kernel
python3 tools/pmc_traffic.py "$OUT/pmc_traffic_n12288.json" "$(first $OUT/pmc12k_FETCH_SIZE '*counter_collection.csv')" \
  "$(first $OUT/pmc12k_WRITE_SIZE '*counter_collection.csv')" "$(first $OUT/trace12k '*kernel_stats.csv')" \
  band_update=syr2k_w band_xm=xm_kernel@xm:12288 pivot_schur=syrk_compact
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "cross_gemm|syrk64l|dgemm8" -f csv -d "$OUT/pmc_mfma" -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-large-n --no-e2e > "$OUT/pmc_mfma.log" 2>&1
echo "pmc mfma done"
python3 tools/mfma_busy.py "$(first $OUT/pmc_mfma '*counter_collection.csv')" "$OUT/pmc_mfma_busy.json" \
  syrk64l=syrk64l cross_gemm=cross_gemm dgemm8=dgemm8
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
python3 tools/stall_passes.py "$OUT/counters.txt" > "$OUT/stall_passes.txt"
i=0
while read -r P; do
  i=$((i + 1))
  N=12288 ROWS=2 REPS=1 timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$LRE" -f csv \
    -d "$OUT/stall$i" -o run -- python3 tools/solve_time.py > "$OUT/stall$i.log" 2>&1
  echo "stall pass $i done"
done < "$OUT/stall_passes.txt"
python3 tools/stall_summary.py "$OUT/stall_n12288.json" band_xm=xm_kernel band_update=syr2k_w \
  pivot_schur=syrk_compact -- $(find "$OUT" -path '*stall*' -name '*counter_collection.csv' | sort)
if [ -z "$SKIP_BENCH" ]; then  # SKIP_BENCH=1: profiles only
  timeout -k 10 900 python3 bench.py > "$OUT/bench.log" 2>&1
  tail -c 3000 "$OUT/bench.log"
fi
