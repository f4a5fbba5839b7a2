#!/bin/bash
# Round-5 GPU check: a chosen subset of the -m gpu tests (TESTS, default the co-residency and
# the files this change touches), then the bench and smoke (TAG names the outputs).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05}
timeout -k 10 ${TT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
if [ -n "$BENCH" ]; then
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
fi
echo ok
