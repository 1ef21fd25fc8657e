#!/bin/bash
# Run the GPU steps listed in a file (one shell command per line, each with
# its own timeout) in order.  A step that exits 0 or 1 (tests that fail)
# lets the next one run; any other status (time limit, abort, segfault, GPU
# fault) ends the call there.   tools/steps.sh FILE
while IFS= read -r cmd; do
  [ -z "$cmd" ] && continue
  case "$cmd" in \#*) continue ;; esac
  echo "[steps] $cmd"
  bash -c "$cmd"
  rc=$?
  if [ $rc -gt 1 ]; then
    echo "[steps] stopped: status $rc"
    exit $rc
  fi
done < "$1"
echo "[steps] done"
