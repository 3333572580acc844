#!/bin/bash
# Round-5 session 36: epoch-priority variants again with the statistics
# snapshots (the fold chain is shorter now): batch K3 A/B.
set -o pipefail
bash tools/k3_ab.sh ${1:-r5s36}ab main noeprio eprio4 eprio2 || exit 1
