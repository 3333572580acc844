#!/bin/bash
# Round-5 session 21: lossless after the one-pass clustering: GPU lossless
# tests, the line, solo kernel stats, HBM bytes.
set -o pipefail
bash tools/gpu_session.sh ${1:-r5s21} ltests lossless lprof1 lpmc || exit 1
