#!/bin/bash
# Round profile: kernel trace + stats over bench.py, then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE) on the bulge chase and the two streaming
# band-reduction kernels (X/M and the rank-64 update), then the per-class traffic JSON, then the default
# bench line (with the CPU baseline).  Every GPU step has its own limit and
# the steps are chained, so the first failure ends the script.
# usage: tools/profile_round.sh OUTDIR [KERNEL_REGEX]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/${1:-gpurun_out/prof}
KRE=${2:-bulge_lds_kernel|syr2k_w_kernel|xm_kernel}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-large-n > "$OUT/trace_bench.log" 2>&1
echo "trace done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$KRE" -f csv -d "$OUT/pmc_$C" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-syrk --no-large-n > "$OUT/pmc_$C.log" 2>&1
  echo "pmc $C done"
done
STATS=$(find "$OUT/trace" -name '*kernel_stats.csv' | sort | sed -n 1p)
FC=$(find "$OUT/pmc_FETCH_SIZE" -name '*counter_collection.csv' | sort | sed -n 1p)
WC=$(find "$OUT/pmc_WRITE_SIZE" -name '*counter_collection.csv' | sort | sed -n 1p)
python3 tools/pmc_traffic.py "$OUT/pmc_traffic.json" "$FC" "$WC" "$STATS" \
  bulge_chase=bulge_lds_kernel band_update=syr2k_w_kernel band_xm=xm_kernel
timeout -k 10 600 python3 bench.py > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log"
