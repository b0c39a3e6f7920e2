bash scripts/gpu_session.sh \
 "r03zd_ab_guards:700:python scripts/variant_ab.py run 5 canonical"
