#!/bin/bash
# Round-5 session 22: k_vp8l_match with XCD-contiguous rows (lossless tests,
# HBM bytes, solo stats), then K3 priority variants A/B.
set -o pipefail
bash tools/gpu_session.sh ${1:-r5s22} ltests lprof1 lpmc || exit 1
bash tools/k3_ab.sh ${1:-r5s22}ab main eprio3 eprio4 lead3 || exit 1
