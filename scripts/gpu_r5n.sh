export TMPDIR=/tmp; mkdir -p gpurun_out/r5n
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -k "slv or ShortLastVoting or short" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r5n/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r5n/pytest.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_ab.sh r5n slv base libpsg || exit $?
