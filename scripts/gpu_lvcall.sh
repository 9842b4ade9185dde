timeout -k 10 400 python3 -u -m pytest tests -m gpu -q -x -k "otr or golden or sampled" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/otr_t.log 2>&1; rc=$?; tail -2 gpurun_out/otr_t.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_ab_bench.sh ab_otr6 libpsg_base libpsg libpsg_base libpsg
