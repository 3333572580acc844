#!/bin/bash
# Round-5 session 23: K3 compiler scheduling strategies and the barrier's
# last-arriver skip, A/B on one box.
set -o pipefail
bash tools/k3_ab.sh ${1:-r5s23}ab main silp smem sbias noskip || exit 1
