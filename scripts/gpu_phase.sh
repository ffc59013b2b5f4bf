#!/bin/bash
# A/B timing of kernel variants plus per-phase cycle counters (phase* builds)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/phase
mkdir -p $O
for v in ${VARIANTS:-base phase}; do
  DGEN_PHASE_PROF=1 DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 400 python bench.py --no-cpu --config ${CFG:-ca_res_storage} --agents ${AGENTS:-200000} --steps 3 --warmup 1 > $O/bench_$v.log 2>&1; rc=$?
  echo "$v rc=$rc $(python -c "import json;d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]);print(round(d['value']), {k:round(v,2) for k,v in d['roofline']['kernel_ms'].items() if isinstance(v,float)})" 2>&1 | tail -1)"
  grep phase_cycles $O/bench_$v.log || true
  case $rc in 0) ;; *) exit $rc;; esac
done
