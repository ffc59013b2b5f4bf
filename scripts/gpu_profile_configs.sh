#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the bench on the other
# BASELINE configurations at 200k agents per GPU: C2 CA-like PV+storage
# (net billing) and C4 extension mode (commercial, demand charges, battery).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
for cfg in ${CONFIGS:-ca_res_storage com_dc_batt}; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$cfg -o run -- python3 bench.py --config $cfg --agents 200000 --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/prof_${TAG}_$cfg.log 2>&1; rc=$?
  echo "$cfg rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": {[^}]*}\|"cpu_baseline": {"value": [0-9.]*' gpurun_out/prof_${TAG}_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
