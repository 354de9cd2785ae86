#!/bin/bash
# One GPU session: steps given as arguments, each a named shell command run under its
# own time limit, in order. A step that fails by assertion (exit 1: a failed test, a
# parity mismatch) is reported and the session goes on; any other failure (a fault,
# abort 134, segfault 139, time limit 124/137) ends the session there.
# usage: gpu_session.sh TAG "name:seconds:command" ...   -> gpurun_out/TAG/<name>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
O=gpurun_out/$TAG; mkdir -p "$O"
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  tail -4 "$O/$name.log" | cut -c1-300
  echo "rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
done
echo "session done"
