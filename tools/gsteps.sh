#!/bin/bash
# Run GPU steps in order, each under its own time limit:
#   bash tools/gsteps.sh "<seconds> <command>" ...
# A step that fails with exit 1 (pytest: test failures) does not stop the chain; any other
# non-zero status (fault, abort 134, segfault 139, time limit 124/137) ends the call there.
for step in "$@"; do
  t=${step%% *}; c=${step#* }
  echo "[gsteps] start ($t s): $c"
  timeout -k 10 "$t" bash -c "$c"
  rc=$?
  echo "[gsteps] rc=$rc: $c"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
