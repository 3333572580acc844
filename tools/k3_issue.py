"""K3 vector-issue roofline from committed rocprofv3 SQ passes.

usage: python tools/k3_issue.py <dir with sq1/ sq2/ sq3/> <out.json> [kernel substring]

Per launch of the kernel (the passes each profile the same bench command;
every launch of the kernel in a pass is averaged): SQ_INSTS_VALU,
SQ_THREAD_CYCLES_VALU (lane utilisation), SQ_WAIT_ANY / SQ_WAVE_CYCLES,
GRBM_GUI_ACTIVE (summed over the 8 XCDs: effective clock = GRBM / 8 /
kernel time, MI355X_MICROARCH.md 'DVFS give-back'), the launch's duration
in each pass, and the issue fraction SQ_INSTS_VALU / (SIMDs x 0.5 x clock x
time): a wave64 VALU instruction holds a SIMD-32 for 2 cycles, so one SIMD
issues at most 0.5 wave-instructions per cycle (MI355X_MICROARCH.md, Wave
scheduling)."""
import collections
import csv
import json
import os
import sys

SIMDS = 256 * 4


def per_launch(path, kernel):
    vals = collections.defaultdict(list)
    durs = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        durs[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return ({k: sum(v) / len(v) for k, v in vals.items()},
            sum(durs.values()) / len(durs), len(durs), r_name(path, kernel))


def r_name(path, kernel):
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            return r["Kernel_Name"]
    return kernel


def main():
    d, out = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_encode<"
    c = {}
    passes = {}
    for p in ("sq1", "sq2", "sq3"):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if os.path.exists(f):
            v, t, n, name = per_launch(f, kernel)
            c.update(v)
            passes[p] = {"launches": n, "avg_duration_s": t}
    t2 = passes["sq2"]["avg_duration_s"]
    clock = c["GRBM_GUI_ACTIVE"] / 8 / t2
    t1 = passes["sq1"]["avg_duration_s"]
    res = {
        "kernel": name, "source": d, "passes": passes,
        "per_launch": {k: c[k] for k in sorted(c)},
        "effective_clock_hz": clock,
        "valu_per_launch": c["SQ_INSTS_VALU"],
        "issue_frac_profiled": c["SQ_INSTS_VALU"] / (SIMDS * 0.5 * clock * t1),
        "lane_utilisation": c.get("SQ_THREAD_CYCLES_VALU", 0) / (64 * c["SQ_INSTS_VALU"]),
        "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
        "note": "issue_frac = SQ_INSTS_VALU / (1024 SIMDs x 0.5 x clock x duration); clock from "
                "GRBM_GUI_ACTIVE / 8 over the sq2 pass's duration; profiled passes run a "
                "lower clock than unprofiled ones (bench.py applies the VALU count and clock "
                "to its own measured duration)",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
