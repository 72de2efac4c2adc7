#!/bin/bash
# Submit one gpurun call; if the pool has no free box (gpurun exit 3: nothing ran,
# nothing charged) wait and submit the same call again, up to 20 times.  Any other
# outcome (success, failure, refusal) is final -- a GPU step that ran is never re-run.
# usage: tools/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then echo "rc=$rc" >> "$log"; exit $rc; fi
  if grep -q "charged=[1-9]" "$log"; then echo "rc=$rc (charged transient)" >> "$log"; exit $rc; fi
  sleep 150
done
echo "gave up after 20 attempts" >> "$log"
