#!/bin/bash
# Profiling session: kernel trace + stats of the default bench command, then
# one PMC pass per counter group on the same 1M-agent workload (2 timed steps).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
AGENTS=${AGENTS:-1000000}
PMC_BENCH="bench.py --agents $AGENTS --steps 2 --warmup 1 --no-cpu"
stop() { case "$1" in 0) return 0;; 124|134|137|139) echo "STOP: exit $1"; exit "$1";; *) echo "(non-fatal exit $1)"; return 0;; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  case $rc in 0|1) ;; *) echo STOP; exit $rc;; esac
fi
if [ "${SKIP_TRACE:-0}" != "1" ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_trace -o run -- python3 bench.py > gpurun_out/prof_${TAG}_trace.log 2>&1; rc=$?
  echo "trace rc=$rc"; tail -1 gpurun_out/prof_${TAG}_trace.log | cut -c1-400; stop $rc
fi
for grp in ${PMC_GROUPS:-"FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum"}; do
  name=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/prof_${TAG}_pmc_$name -o run -- python3 $PMC_BENCH > gpurun_out/prof_${TAG}_pmc_$name.log 2>&1; rc=$?
  echo "pmc $grp rc=$rc"; stop $rc
done
python3 scripts/pmc_summary.py $TAG $AGENTS > gpurun_out/prof_${TAG}_pmc_summary.txt 2>&1; cat gpurun_out/prof_${TAG}_pmc_summary.txt
