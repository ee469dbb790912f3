"""Print the dispatch timeline (ms) of a rocprofv3 kernel trace: python tools/timeline.py trace.csv [min_ms]"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
# last frame only: from the last k_iow03 spec first-pass launch burst
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if d > lim:
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e6:10.1f} {d:10.2f} {r['Kernel_Name'][:60]}")
