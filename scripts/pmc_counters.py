"""Per-kernel mean PMC counter values per dispatch from rocprofv3 --pmc passes
(run_counter_collection.csv files) -> JSON {kernel: {counter: mean, dispatches}}.

    python scripts/pmc_counters.py OUT.json DIR1 [DIR2 ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def main(out, dirs):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    acc[short(row["Kernel_Name"])][row["Counter_Name"]][row["Dispatch_Id"]] += \
                        float(row["Counter_Value"])
    res = {}
    for k, cs in sorted(acc.items()):
        res[k] = {c: sum(v.values()) / len(v) for c, v in sorted(cs.items())}
        res[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump({"meta": {"source": dirs, "value": "mean per dispatch, summed over XCDs/SEs"},
               "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k, {c: round(x, 1) for c, x in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
