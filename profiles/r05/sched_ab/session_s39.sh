# round-5 session 39: scheduler A/B for the hourly scan (max-ilp, max-memory-clause; whole library) on C3 and C2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TAG=r05/s39
C3="--config res_1m_nem_tou --agents 1000000 --steps 10 --warmup 2 --no-cpu"
C2="--config ca_res_storage --agents 200000 --steps 5 --warmup 1 --no-cpu"
VARIANTS="$C3;lib=ilp $C3;lib=memcl $C3;$C3;$C2;lib=ilp $C2;lib=memcl $C2" bash scripts/gpu.sh ab
