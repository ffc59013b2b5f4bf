#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/tierab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest gpu rc=$rc $(grep -E 'passed|failed' $O/pytest_gpu.log | tail -1)"; case $rc in 0|1) ;; *) exit $rc;; esac
for v in notierskip tierskip notierskip tierskip; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 > $O/$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(python -c "import json;d=json.loads(open('$O/$v.log').read().strip().splitlines()[-1]);print(round(d['value']), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items() if isinstance(v,float)})" 2>&1 | tail -1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
