bash scripts/gpu_ab_cfg.sh ab_eps1 "eps" W2_epsilon libpsg_base libpsg
