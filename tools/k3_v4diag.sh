# K3 worker-variant stall localisation (WEBP_AMD_SYNC_K3 prints each frame's
# raw K3 error: wait site << 4); usage: bash tools/k3_v4diag.sh VARIANT...
export WEBP_AMD_SYNC_K3=1
for var in "$@"; do
for cfg in "64 64" "256 256"; do
  set -- $cfg
  echo "== variant $var ${1}x${2}"
  WEBP_AMD_K3=$var timeout -k 10 100 python -u bench.py --no-cpu --no-host-input --steps 1 --warmup 0 --engines 1 --batch 8 --width $1 --height $2 2>&1 | grep -E "K3 error|metric|Error" | sort | uniq -c | head -4
  rc=${PIPESTATUS[0]}
  echo "rc=$rc"
  if [ "$rc" != 0 ] && [ "$rc" != 1 ]; then exit $rc; fi
done
done
