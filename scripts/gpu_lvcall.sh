bash scripts/gpu_ab_cfg.sh ab_spec2 "spec" G1_lv_n64_fused,G1_otr_n64_fused libpsg && \
PSG_FUSED_WPE=6 timeout -k 10 300 python3 bench_configs.py --only G1_lv_n64_fused,G1_otr_n64_fused --steps 2 --warmup 1 > gpurun_out/ab_spec2/wpe6.log 2>&1 && \
PSG_FUSED_WPE=7 timeout -k 10 300 python3 bench_configs.py --only G1_lv_n64_fused,G1_otr_n64_fused --steps 2 --warmup 1 > gpurun_out/ab_spec2/wpe7.log 2>&1; grep -h '^{' gpurun_out/ab_spec2/wpe*.log | cut -c1-300
