#!/bin/bash
# One eigh_values timing per library variant, each under its own limit
# (development tool): tools/bulge_try.sh lib1.so lib2.so ...  (ENVSTATS=0: no TG_BULGE_STATS)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for so in "$@"; do
  echo "== $so"
  if [ "${ENVSTATS:-1}" = 1 ]; then export TG_BULGE_STATS=1; else unset TG_BULGE_STATS; fi
  TRUNCGPTQ_LIB=$PWD/$so REPS=${REPS:-2} timeout -k 5 ${LIM:-45} python -u tools/eigv_time.py 2>&1 | grep -v amdgpu.ids
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
