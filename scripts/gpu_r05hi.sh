bash scripts/gpu_r05i.sh && bash scripts/gpu_r05h.sh
