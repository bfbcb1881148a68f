#!/bin/bash
# bench (default args, with CPU baseline) + rocprofv3 kernel-trace/stats of a short bench.
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$PYTEST_K" ]; then
  if [ "$PYTEST_K" = "all" ]; then KARG=(); else KARG=(-k "$PYTEST_K"); fi
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf "${KARG[@]}" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench_default.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_default.log
  [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps ${PROF_STEPS:-5} --warmup 2 --no-cpu-baseline --no-nocfg $PROF_ARGS > $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*.csv" | head
exit $rc
