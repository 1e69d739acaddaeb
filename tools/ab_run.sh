# A/B driver for gpurun: optional GPU tests, then tools/ab.sh over the variant list
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
STEPS=${STEPS:-200} EXTRA="--warmup 300 ${EXTRA:-}" bash tools/ab.sh "$@"
