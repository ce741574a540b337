"""Timeline of the last N kernels of a rocprofv3 kernel trace (csv): start
offset, duration and the idle gap before each, to see where a step's time goes."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in rows))[-last:]
t0 = ks[0][0]
prev_end = ks[0][0]
for s, e, name in ks:
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev_end) / 1e3:8.1f}  {name}")
    prev_end = max(prev_end, e)
