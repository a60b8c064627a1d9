"""Keep only the slam355 kernels (and copies) of a rocprofv3 kernel_trace.csv:
name, stream/queue, start, end (ns) -> a small CSV for timeline analysis.

    python scripts/trace_extract.py TRACE_DIR OUT.csv
"""
import csv
import glob
import os
import sys


def main(d, out):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                n = r["Kernel_Name"]
                if "at::native" in n:
                    continue
                n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n,
                             r.get("Queue_Id", ""), r.get("Stream_Id", ""),
                             r.get("Grid_Size_X", r.get("Grid_Size", "")),
                             r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))))
    rows.sort()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["start", "end", "name", "queue", "stream", "grid", "wg"])
        w.writerows(rows)
    print(len(rows), "kernels")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
