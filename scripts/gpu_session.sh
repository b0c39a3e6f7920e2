#!/bin/bash
# One GPU session: steps given as "name:timeout:command" arguments, each under its own time limit.
# A crash/abort/timeout (rc >= 124, or 134/139) ends the session; plain test failures (rc 1) continue.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; t=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($(date +%T))"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
