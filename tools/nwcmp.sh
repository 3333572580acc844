set -e -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/nw
for V in 3 5 4; do
  WEBP_AMD_K3=$V timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/nw/b$V.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
for V in 3 5; do
  WEBP_AMD_K3=$V timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/nw/f$V -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $R/gpurun_out/nw/pf$V.log 2>&1
done
echo done
