bash scripts/gpu_session.sh \
 "r03x_gputest_tiny:300:python -u -m pytest tests/test_gpu_ragged.py -x -q -k 'tiny or info_steps' --timeout 120 --timeout-method thread"
