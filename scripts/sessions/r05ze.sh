S=scripts/gpu_session.sh
$S "r05ze_torchrun_ab:1000:scripts/torchrun_ab.sh r05ze 6 plain:plain busy:torchrun nobusy:torchrun:WG_BENCH_BARRIER_BUSY=0"
