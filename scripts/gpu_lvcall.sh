bash scripts/gpu_ab.sh ab_slv2 W2_slv libpsg libpsg_w6 libpsg_w7
