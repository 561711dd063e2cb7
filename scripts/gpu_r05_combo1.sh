bash scripts/gpu_r05_comm_ab.sh && bash scripts/gpu_r05_gbdt.sh
