bash scripts/gpu_ab.sh ab_ks2 C4_kset libpsg libpsg_ks3 libpsg libpsg_ks3
