#!/bin/bash
# A/B the full bench over library variants (development tool):
#   tools/bench_ab.sh OUT_PREFIX lib1.so lib2.so ...   (each under its own time limit)
set -e
P=$1; shift
i=0
for L in "$@"; do
  TRUNCGPTQ_LIB=$L timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-syrk > "${P}_$i.log" 2>&1
  python3 -c "
import json,sys
d=json.loads(open('${P}_$i.log').read().strip().splitlines()[-1]); print('$L', d['value'], d['ms_per_step'], d['phases_ms'])"
  i=$((i+1))
done
