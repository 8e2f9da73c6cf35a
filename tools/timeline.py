"""Print one step's kernel timeline from a rocprofv3 kernel trace (between two
consecutive launches of a marker kernel, default the request generator)."""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "gen_requests"
skip = () if len(sys.argv) > 3 and sys.argv[3] == "all" else ("fillBuffer",)
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
gens = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
i0, i1 = gens[-3], gens[-2]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    if any(s in r["Kernel_Name"] for s in skip):
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %7.1f  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, r.get("Queue_Id", ""), r["Kernel_Name"][:64]))
