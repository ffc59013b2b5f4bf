#!/bin/bash
# A/B of k_hourly_batt occupancy variants (scripts/make_ablations.py) on the
# default C3 bench: per-kernel ms per step from the bench's HIP events.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/occ
mkdir -p $O
for v in ${VARIANTS:-base hb_w3 hb_w4 base}; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 > $O/$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(python -c "import json;d=json.loads(open('$O/$v.log').read().strip().splitlines()[-1]);print(round(d['value']), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items() if isinstance(v,float)})" 2>&1 | tail -1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
