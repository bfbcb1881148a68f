#!/bin/bash
# GPU round trip: parity tests, then (only if nothing crashed) a short bench.
# Stops on any abnormal exit (fault / abort / timeout); ordinary test failures
# (pytest rc 1) still let the bench run.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf --maxfail=30 ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -8 gpurun_out/bench.log
exit $brc
