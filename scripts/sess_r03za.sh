bash scripts/gpu_session.sh \
 "r03za_ab_canon_res:500:WG_AB_RESIDENT=1 python scripts/variant_ab.py run 3 canonical"
