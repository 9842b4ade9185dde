bash scripts/gpu_ab_cfg.sh ab_lv2 "lv or lastvoting" C3_lastvoting,G1_lv_n64_fused,G1_otr_n64_fused libpsg_base libpsg
