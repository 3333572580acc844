#!/bin/bash
# Round-5 session 16: K3 structure A/B on one box: main (intra-4 || chroma
# fork), no fork, no fork with the compiler's barrier code, round-4's K3.
set -o pipefail
bash tools/k3_ab.sh ${1:-r5s16}ab main nofork noforkv r4 || exit 1
