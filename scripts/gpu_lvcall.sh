bash scripts/gpu_ab.sh ab_lvk C3_lastvoting libpsg libpsg_k1 libpsg_k2
