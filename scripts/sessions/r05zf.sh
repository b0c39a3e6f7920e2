S=scripts/gpu_session.sh
$S "r05zf_torchrun_ab:1000:scripts/torchrun_ab.sh r05zf 6 plain:plain spin:torchrun nospin:torchrun:WG_BENCH_SPIN_US=0"
