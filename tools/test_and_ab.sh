#!/bin/bash
# GPU tests, then an A/B bench of variant libraries (run via gpurun from the repo root):
#   tools/test_and_ab.sh TAG LIB1 LIB2 ...
set -o pipefail
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$TAG.tests.log 2>&1
rc=$?
tail -1 gpurun_out/$TAG.tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab2.sh $TAG "$@" "$@"
