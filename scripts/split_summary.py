"""Per-rank split of the sharded LM iteration (scripts/gpu_r5_split3.sh output):
rocprofv3 kernel averages of each {C4|C5}_w{W}_r{r} run -> divided (k_lin_mfma +
k_asm_fill + k_assemble + k_back_trial) and replicated (k_tl3_flow + k_tl2_load +
k_tl2_scatter) microseconds per LM iteration, plus the run's own wall time per
iteration.   python scripts/split_summary.py OUTDIR > summary.json"""
import csv
import glob
import json
import os
import sys

DIV = ("k_lin_mfma", "k_asm_fill", "k_assemble", "k_back_trial")
REP = ("k_tl3_flow", "k_tl2_load", "k_tl2_scatter")


def main(d):
    res = {}
    for path in sorted(glob.glob(os.path.join(d, "C*_w*_r*", "run_kernel_stats.csv"))):
        name = os.path.basename(os.path.dirname(path))
        avg = {}
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                k = k.split("<")[0]
                if k in DIV + REP:
                    avg[k] = round(float(r["AverageNs"]) / 1e3, 1)
        e = dict(avg)
        e["divided"] = round(sum(avg.get(k, 0.0) for k in DIV), 1)
        e["replicated"] = round(sum(avg.get(k, 0.0) for k in REP), 1)
        js = os.path.join(d, name + ".json")
        if os.path.exists(js):
            try:
                line = json.loads(open(js).read().strip().splitlines()[-1])
                e["wall_us_per_iter"] = round(line["ms_per_iter_alone"] * 1e3, 1)
            except (ValueError, IndexError):
                pass
        res[name] = e
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
