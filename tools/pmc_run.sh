#!/bin/bash
# usage: tools/pmc_run.sh OUTDIR "COUNTERS" cmd...   (run from /tmp with TMPDIR=/tmp)
out=$1; shift; ctr=$1; shift
timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d "$out" -o run -- "$@"
