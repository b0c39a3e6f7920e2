S=scripts/gpu_session.sh
$S "r05zj_split_ab:900:KS='20 5;1000 50' scripts/issue_ab.sh r05zj 3 canonical s50: s60:WG_RANGE_SPLIT=0.6 s67:WG_RANGE_SPLIT=0.67 s40:WG_RANGE_SPLIT=0.4"
