S=scripts/gpu_session.sh
$S "r05zh_plain_spin_ab:900:scripts/torchrun_ab.sh r05zh 8 plain:plain pspin:plain:WG_BENCH_SPIN_PLAIN=300"
