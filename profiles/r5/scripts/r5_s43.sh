#!/bin/bash
# Round-5 session 43: the 16-bit overflow check every 32 columns (threshold
# 0xc000) instead of 16 (0xe000): early-fold test, parity subset, K3 A/B.
set -o pipefail
O=gpurun_out/${1:-r5s43}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_early_fold.py \
  tests/test_gpu_parity.py tests/test_token_fallbacks.py tests/test_multipass.py tests/test_shards.py \
  > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/k3_ab.sh ${1:-r5s43}ab main every16 || exit 1
