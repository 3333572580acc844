#!/bin/bash
# Round-5 session 20: epoch-boundary priority + branch-free token count as
# the default: GPU suite, A/B against no priority and a three-level variant.
set -o pipefail
O=gpurun_out/${1:-r5s20}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  > $O/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/k3_ab.sh ${1:-r5s20}ab main noeprio eprio2 || exit 1
