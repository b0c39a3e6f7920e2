S=scripts/gpu_session.sh
$S "r05l_ab_nolast:500:python scripts/variant_ab.py run 5 canonical && cp gpurun_out/variant_ab_canonical.json gpurun_out/r05l_ab_nolast.json" \
   "r05l_ab_obsalign:500:WG_AB_ONLY=none python scripts/variant_ab.py run 5 ragged al0: al32:WG_OBS_ALIGN=32 && cp gpurun_out/variant_ab_ragged.json gpurun_out/r05l_ab_obsalign.json"
