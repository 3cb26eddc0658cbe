#!/bin/bash
# tg_band_tridiag per library variant under its own limit (development tool)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for so in "$@"; do
  echo "== $so"
  TRUNCGPTQ_LIB=$PWD/$so timeout -k 5 ${LIM:-45} python -u tools/bulge_check.py > gpurun_out/one.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/one.log
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
