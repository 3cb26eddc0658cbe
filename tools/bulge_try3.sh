#!/bin/bash
# tg_band_tridiag per library variant, each under its own limit; continues
# past a hang (development tool)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for so in "$@"; do
  echo "== $so"
  TRUNCGPTQ_LIB=$PWD/$so timeout -k 5 ${LIM:-30} python -u tools/bulge_check.py > gpurun_out/one.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/one.log | head -12
  echo "rc=$rc"
  case $rc in 134|139) exit $rc;; esac
done
