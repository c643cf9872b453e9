"""Print a rocprofv3 kernel_stats.csv sorted by total time (short names):
python tools/kstats.py path/to/run_kernel_stats.csv [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    name = r["Name"].replace("void ", "").replace("ctr::", "")
    name = name.split("(")[0][:80]
    print(f"{float(r['TotalDurationNs']) / 1e3:10.1f} us  {int(r['Calls']):5d} calls  "
          f"{float(r['AverageNs']) / 1e3:8.2f} us/call  {name}")
