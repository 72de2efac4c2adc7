#!/bin/bash
# ResNet-50 --graph capture: which call invalidates the capture (HIP API log)
mkdir -p gpurun_out
run() { local name=$1; shift; echo "=== $name: $*"; timeout -k 10 240 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; grep -a "CAPTURE" gpurun_out/$name.log | head -3; return $rc; }
run gplain python -u tools/graph_debug.py plain &&
run gstem_relaxed env CAPTURE_MODE=relaxed python -u tools/graph_debug.py stem &&
run gstem_noamp env NO_AMP=1 python -u tools/graph_debug.py stem &&
run gstem_log env AMD_LOG_LEVEL=4 python -u tools/graph_debug.py stem
rc=$?
# keep only the part of the API log around the capture
if [ -f gpurun_out/gstem_log.log ]; then
  grep -an "BeginCapture\|hipStreamBeginCapture\|Invalidated\|hipErrorStreamCapture\|EndCapture" gpurun_out/gstem_log.log | head -40 > gpurun_out/gstem_log_marks.txt
  first=$(grep -an "hipStreamBeginCapture" gpurun_out/gstem_log.log | tail -1 | cut -d: -f1)
  if [ -n "$first" ]; then sed -n "${first},$((first+400))p" gpurun_out/gstem_log.log > gpurun_out/gstem_log_capture.txt; fi
  gzip -f gpurun_out/gstem_log.log
fi
exit $rc
