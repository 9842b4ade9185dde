bash scripts/gpu_ab_cfg.sh ab_spec1 "spec" G1_lv_n64_fused,G1_otr_n64_fused,G1_lv_n64_native libpsg
