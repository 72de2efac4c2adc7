#!/bin/bash
# GPU session driver: each GPU step has its own timeout; a crash/abort/timeout
# (exit >= 2 other than pytest's 1 = test failures) ends the session.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1; local to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL step $name rc=$rc -- stopping"; exit $rc; fi
  return 0
}
for s in "$@"; do
  eval "$s" || exit $?
done
