S=scripts/gpu_session.sh
$S "r05zd_torchrun_ab:900:scripts/torchrun_ab.sh r05zd 6"
