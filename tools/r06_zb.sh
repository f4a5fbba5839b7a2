#!/bin/bash
# the default bench line at the final sources, after the PMC passes were committed under
# profiles/ (bench.py fills roofline.traffic from them when their csrc hash matches)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG:-r06z}_bench.json 2> gpurun_out/${TAG:-r06z}_bench.err
echo ok
