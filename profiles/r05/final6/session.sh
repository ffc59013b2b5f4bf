# round-5 session 37: search kernels in their own translation unit (iterative max-occupancy scheduler) -- full GPU suite, smoke, bench lines, C3 trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TAG=r05/s37
bash scripts/gpu.sh tests smoke || exit 1
bash scripts/gpu.sh bench || exit 1
BENCH="ca_res_storage:200000:--steps,5,--warmup,1,--no-cpu national_mixed:200000:--steps,5,--warmup,1,--no-cpu com_dc_batt:200000:--steps,5,--warmup,1,--no-cpu com_dc_batt:1000000:--steps,5,--warmup,1,--no-cpu" bash scripts/gpu.sh bench || exit 1
LOOP_ARGS="--agents 2500000 --hourly-chunk 500000 --years 25" LOOP_TIMEOUT=600 bash scripts/gpu.sh loop || exit 1
PROF="res_1m_nem_tou:1000000" bash scripts/gpu.sh trace
