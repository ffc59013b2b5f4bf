# round-5 session 36: compiler-scheduler A/B (AMDGPU trackers, iterative min-reg / max-occupancy) on C3, C2, C4
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TAG=r05/s36
C3="--config res_1m_nem_tou --agents 1000000 --steps 10 --warmup 2 --no-cpu"
C2="--config ca_res_storage --agents 200000 --steps 5 --warmup 1 --no-cpu"
C4="--config com_dc_batt --agents 200000 --steps 5 --warmup 1 --no-cpu"
VARIANTS="$C3;lib=trk $C3;lib=minreg $C3;lib=maxocc $C3;$C2;lib=trk $C2;lib=minreg $C2;lib=maxocc $C2;$C4;lib=trk $C4;lib=minreg $C4;lib=maxocc $C4;$C3" bash scripts/gpu.sh ab
