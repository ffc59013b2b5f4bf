#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AGENTS=${AGENTS:-200000}
for v in base no_target no_hourly_stores no_bins; do
  DGEN_LIB=$PWD/dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python bench.py --agents $AGENTS --steps 5 --warmup 1 --no-cpu > gpurun_out/ablate_$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/ablate_$v.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])" 2>&1 | tail -1)"
  case $rc in 0) ;; *) echo STOP; exit $rc;; esac
done
