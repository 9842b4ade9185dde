bash scripts/gpu_round.sh r3b && bash scripts/gpu_ab_probe.sh ab_lv3 "" "C3,G1_otr_n64_fused,G1_lv_n64_fused" lib_lv2 lib_lv3
