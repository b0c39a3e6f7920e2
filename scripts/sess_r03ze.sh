bash scripts/gpu_session.sh \
 "r03ze_ab_guards:700:python scripts/variant_ab.py run 7 canonical"
