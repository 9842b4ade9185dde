bash scripts/gpu_ab.sh ab_wpe C3_lastvoting,W2_epsilon libpsg_base libpsg_lv7 libpsg_e6 libpsg_e7
