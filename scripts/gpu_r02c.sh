#!/bin/bash
# Round-2 GPU session C: is the spilling two-agent DC miscompile the VGPR
# live-range optimisation?  Same builds with -amdgpu-opt-vgpr-liverange=false.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
ok() { case "$1" in 0|1) return 0;; *) echo "STOP: exit $1"; exit "$1";; esac; }
DGEN_LIB=dgen_amd/lib/ablate/libdgen_dc2w_nolr.so timeout -k 10 300 python -u -m pytest tests/test_gpu_demand.py -q --timeout 120 --timeout-method thread > $O/pytest_dc2w_nolr.log 2>&1; rc=$?
echo "dc2w_nolr rc=$rc"; tail -3 $O/pytest_dc2w_nolr.log; ok $rc
for v in good_nolr bad_nolr; do
  DGEN_LIB=dgen_amd/lib/ablate/libdgen_dbg_$v.so timeout -k 10 200 python -u scripts/dbg_dc_dump.py $O/dc_$v.npz > $O/dump_$v.log 2>&1; rc=$?
  echo "dump $v rc=$rc"; ok $rc
done
python scripts/dbg_dc_compare.py $O/dc_good_nolr.npz $O/dc_bad_nolr.npz | tee $O/compare.log
python -c "
import numpy as np
for v in ('good_nolr','bad_nolr'):
    a=np.load('$O/dc_'+v+'.npz'); print(v, 'npv nan', int(np.isnan(a['npv']).sum()), a['npv'][:3], a['nfev'][:6], a['cash_flow'][0][:3])
"
