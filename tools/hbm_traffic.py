"""profiles/hbm_traffic.json from one session's rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE, one counter per pass, bench.py --steps 1
--warmup 0 of the default workload). rocprofv3 reports both in KiB. gfx950
correction (profiles/r2/calib_*: a 1 GiB stream of dword / dwordx4 loads
reads back as 0.5 GiB of FETCH_SIZE, 1 GiB of stores as 1 GiB of
WRITE_SIZE): FETCH_SIZE x 2, WRITE_SIZE as is.

usage: python tools/hbm_traffic.py gpurun_out/<tag> [workload text] > profiles/hbm_traffic.json"""
import collections
import csv
import json
import os
import sys


def load(path):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        out[name].append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    d = sys.argv[1]
    workload = sys.argv[2] if len(sys.argv) > 2 else "256 x 1920x1080 q75 m4"
    fetch = load(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        if name.startswith("__amd") or "at::native" in name or name == "k_synth":
            continue
        f = sum(fetch.get(name, [0.0])) / max(1, len(fetch.get(name, [1])))
        w = sum(write.get(name, [0.0])) / max(1, len(write.get(name, [1])))
        short = name.replace("void ", "").split("<")[0]
        kernels[short if short not in kernels else name] = {
            "fetch_bytes_raw": int(f), "fetch_bytes": int(2 * f), "write_bytes": int(w),
            "bytes_per_launch": int(2 * f + w)}
    json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                         "bench.py --steps 1 --warmup 0 (%s), "
                         "FETCH_SIZE x2 (gfx950 calibration profiles/r2/calib_*)" % workload,
               "session": os.path.basename(os.path.normpath(d)),
               "kernels": kernels}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
