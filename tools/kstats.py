"""Print the top kernels of a rocprofv3 --stats CSV (kernel_stats.csv)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:n]:
    print('%-58s %6s %10.1f us  avg %8.2f  %5.1f%%' % (r['Name'][:58], r['Calls'], float(r['TotalDurationNs']) / 1e3,
                                                     float(r['AverageNs']) / 1e3, 100 * float(r['TotalDurationNs']) / tot))
