mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/t1.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/t1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --instances 2000000 --cpu-seconds 5 > gpurun_out/b1.log 2>&1; echo "bench rc=$?"; tail -3 gpurun_out/b1.log
fi
