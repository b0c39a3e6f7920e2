S=scripts/gpu_session.sh
$S "r05zn_degree_lpt2:600:python scripts/degree_sort_ab.py 7 200 && cp gpurun_out/degree_sort_ab.json gpurun_out/r05zn_degree_sort_lpt2.json"
