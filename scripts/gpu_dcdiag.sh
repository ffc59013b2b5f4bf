#!/bin/bash
# Demand-charge two-agent k_size diagnosis: the parity test (NEM, two agents
# per wave) against each variant library of scripts/make_ablations.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/dcdiag
mkdir -p $O
for v in ${VARIANTS:-base dc_rel dc_noenv dc_noeval}; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_demand.py -m gpu -q -s \
    -k "False-False or True-False" --timeout 120 --timeout-method thread > $O/$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(grep -E 'passed|failed' $O/$v.log | tail -1) $(grep -o 'AssertionError: ([^)]*)' $O/$v.log | head -2 | tr '\n' ' ')"
  case $rc in 0|1) ;; *) echo STOP; exit $rc;; esac
done
