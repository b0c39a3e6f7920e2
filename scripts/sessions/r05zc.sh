S=scripts/gpu_session.sh
$S "r05zc_degree_lpt:600:python scripts/degree_sort_ab.py 5 200 && cp gpurun_out/degree_sort_ab.json gpurun_out/r05zc_degree_sort_lpt.json"
