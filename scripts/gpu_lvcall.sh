bash scripts/gpu_ab_cfg.sh ab_lvs2 "lv or lastvoting" C3_lastvoting,G1_lv_n64_fused libpsg
