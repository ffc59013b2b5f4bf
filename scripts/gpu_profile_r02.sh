#!/bin/bash
# Round-2 profiling session: per workload, the rocprofv3 kernel trace + stats
# of its bench command and one PMC pass per counter group (each pass its own
# run), summarised into gpurun_out/r02p/pmc_<workload>.json.
#   WORKLOADS="config:agents ..."  (default: C3 1M, C2 200k, C4 200k)
#   LOOP=1 also profiles the national model-year loop (C5) at LOOP_AGENTS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r02p
mkdir -p $O
stop() { case "$1" in 0) return 0;; 124|134|137|139) echo "STOP: exit $1"; exit "$1";; *) echo "(exit $1)"; return 0;; esac; }
GROUPS_=("FETCH_SIZE" "WRITE_SIZE"
         "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
         "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY")
cd /tmp
WL=${WORKLOADS:-res_1m_nem_tou:1000000 ca_res_storage:200000 com_dc_batt:200000}
for wa in $WL; do
  W=${wa%%:*}; A=${wa##*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- \
    python3 $R/bench.py --config $W --agents $A --steps 5 --warmup 1 --no-cpu > $O/trace_$W.log 2>&1; rc=$?
  echo "trace $W rc=$rc"; stop $rc
  for grp in "${GROUPS_[@]}"; do
    name=$(echo $grp | cut -d' ' -f1)
    timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${W}_$name -o run -- \
      python3 $R/bench.py --config $W --agents $A --steps 2 --warmup 1 --no-cpu > $O/pmc_${W}_$name.log 2>&1; rc=$?
    echo "pmc $W $name rc=$rc"; stop $rc
  done
  python3 $R/scripts/pmc_summary.py "$O/pmc_${W}_*" $A $O/pmc_$W.json > $O/pmc_$W.txt 2>&1
  head -4 $O/pmc_$W.txt
done
if [ -n "$LOOP" ]; then
  LA=${LOOP_AGENTS:-1000000}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loop -o run -- \
    python3 $R/bench_loop.py --agents $LA --years 3 > $O/trace_loop.log 2>&1; rc=$?
  echo "trace loop rc=$rc"; stop $rc
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_loop_$grp -o run -- \
      python3 $R/bench_loop.py --agents $LA --years 2 > $O/pmc_loop_$grp.log 2>&1; rc=$?
    echo "pmc loop $grp rc=$rc"; stop $rc
  done
  python3 $R/scripts/pmc_summary.py "$O/pmc_loop_*" $LA $O/pmc_national_loop.json > $O/pmc_loop.txt 2>&1
  head -4 $O/pmc_loop.txt
fi
