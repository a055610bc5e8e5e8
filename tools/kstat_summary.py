"""Print a rocprofv3 kernel_stats.csv as name / calls / average us / share (names without argument lists)."""
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("insfm::", "")
    return re.split(r"\(", name, maxsplit=1)[0]


for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        print(f"{short(r['Name'])[:44]:44s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1000:8.2f} us"
              f"  {float(r['Percentage']):5.2f} %")
