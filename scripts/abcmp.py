"""Per-kernel comparison of two rocprofv3 --stats runs (ms per step, 4 calls per step-equivalent)."""
import csv
import sys


def load(p, div):
    d = {}
    for r in csv.DictReader(open(p)):
        n = r['Name'].replace('void (anonymous namespace)::', '').replace('(anonymous namespace)::', '')[:90]
        d[n] = d.get(n, 0) + float(r['TotalDurationNs']) / 1e6 / div
    return d


a, b = sys.argv[1], sys.argv[2]
div = float(sys.argv[3]) if len(sys.argv) > 3 else 4.0
x, y = load(a + '/run_kernel_stats.csv', div), load(b + '/run_kernel_stats.csv', div)
print("total base %.1f new %.1f ms/step" % (sum(x.values()), sum(y.values())))
for k in sorted(set(x) | set(y), key=lambda k: -abs(y.get(k, 0) - x.get(k, 0)))[:int(sys.argv[4]) if len(sys.argv) > 4 else 25]:
    print("%8.2f %8.2f %+7.2f %s" % (x.get(k, 0), y.get(k, 0), y.get(k, 0) - x.get(k, 0), k))
