S=scripts/gpu_session.sh
$S "r05u_ab_stagger:600:python scripts/variant_ab.py run 5 canonical && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05u_ab_stagger_canonical.json"
