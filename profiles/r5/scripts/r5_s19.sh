#!/bin/bash
# Round-5 session 19: K3 options A/B on the final base (next-MB prefetch,
# epoch-boundary priority, branch-free token count, all three); then the
# lossless line, its kernel stats and HBM bytes.
set -o pipefail
bash tools/k3_ab.sh ${1:-r5s19}ab main pf eprio cnt all3 || exit 1
bash tools/gpu_session.sh ${1:-r5s19} lossless lprof1 lpmc || exit 1
