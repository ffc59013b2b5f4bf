#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/dcdiag
mkdir -p $O
VARIANTS=dc_dbg bash scripts/gpu_dcdiag.sh || exit $?
DGEN_LIB=dgen_amd/lib/ablate/libdgen_dc_dbg.so timeout -k 10 300 python -u scripts/dbg_dc_eval.py > $O/dc_dbg_eval.log 2>&1; rc=$?
echo "dbg rc=$rc"; head -60 $O/dc_dbg_eval.log
