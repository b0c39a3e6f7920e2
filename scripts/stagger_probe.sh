cd "${GRAFT_REPO_ROOT:-/root/repo}"
for st in 0 4 16 64; do echo "stagger $st: $(WG_STAGGER=$st WG_STREAM=0 timeout -k 10 100 python scripts/ablate.py one walker_gym_amd/libwalker_hip.so 2>/dev/null)"; done
for n in 4096 8192 16384; do echo "N $n: $(WG_N=$n WG_STREAM=0 timeout -k 10 100 python scripts/ablate.py one walker_gym_amd/libwalker_hip.so 2>/dev/null)"; done
