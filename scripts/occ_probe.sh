cd "${GRAFT_REPO_ROOT:-/root/repo}"
for x in 0 8192 12288 24000; do echo "extra $x: $(WG_DEBUG_LDS_EXTRA=$x timeout -k 10 100 python scripts/sweep_w.py one 2>/dev/null)"; done
