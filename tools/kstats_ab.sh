#!/bin/bash
# Per-kernel averages of tg_eigh_values (tools/eigv_time.py) per library
# variant, from rocprofv3 kernel-trace stats (development tool).
#   tools/kstats_ab.sh lib_a.so lib_b.so ...   (KRE: kernel-name regex to print)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
KRE=${KRE:-syr2k_bs|dgemm_chunked|pqr_kernel|ytx_m|splitk_reduce|bulge_lds}
i=0
for so in "$@"; do
  D=gpurun_out/ks_$i
  echo "== $so"
  TRUNCGPTQ_LIB=$R/$so REPS=${REPS:-4} timeout -k 10 ${LIM:-120} rocprofv3 --kernel-trace --stats \
    -f csv -d "$D" -o run -- python3 tools/eigv_time.py > "$D.log" 2>&1 || { echo "rc=$?"; tail -5 "$D.log"; exit 1; }
  grep eigh_values "$D.log"
  S=$(find "$D" -name '*kernel_stats.csv' | sort | sed -n 1p)
  python3 - "$S" "$KRE" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print(f'  {r["Name"][:70]:70s} calls {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e3:8.2f} us total {float(r["TotalDurationNs"])/1e6:8.2f} ms')
PY
  i=$((i+1))
done
