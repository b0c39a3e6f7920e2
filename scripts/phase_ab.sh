# Per-step time (config 2 by default; WG_WORKLOAD / WG_N / PHASE_ARGS for others) along a 1,500-step Balance-v0 rollout, per A/B library (scripts/balance_phase.py), interleaved
set -e
for r in 1 2; do
  for v in ${PHASE_LIBS:-nodead dead}; do
    WALKER_HIP_LIB=ab_session/lib_$v.so timeout -k 10 120 python scripts/balance_phase.py ${PHASE_ARGS:-1500 100 1} > /dev/null
    cp gpurun_out/balance_phase.json gpurun_out/balance_phase_${v}_$r.json
    echo "$v $r $(python -c "import json; d=json.load(open('gpurun_out/balance_phase.json')); print([r['us_per_step'] for r in d['runs']['1.0']])")"
  done
done
