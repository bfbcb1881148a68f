#!/bin/bash
# Round checkpoint: all GPU tests, the default bench line, then rocprof step breakdowns at
# 16 and 2 frames (tools/prof_frames.sh).  Stops at the first abnormal exit.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit 1
cat gpurun_out/bench_default.json
[ -n "$NO_PROF" ] && exit $rc
bash tools/prof_frames.sh || exit 1
exit $rc
