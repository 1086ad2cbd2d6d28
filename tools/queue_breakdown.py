"""Per-queue kernel time of the last bench step in a rocprofv3 kernel trace (steps delimited by
embed_fwd_kernel launches), grouped by kernel (name + grid).  Usage:
python tools/queue_breakdown.py <prof dir> [queue] [top]"""
import csv
import re
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
want_q = int(sys.argv[2]) if len(sys.argv) > 2 else None
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     r["Kernel_Name"], int(r["Grid_Size_X"])))
rows.sort()
starts = [i for i, r in enumerate(rows) if "embed_fwd_kernel" in r[3]]
a, b = starts[-2], starts[-1]
step = rows[a:b]
t0, t1 = step[0][0], step[-1][1]
tot = defaultdict(float)
cnt = defaultdict(int)
qt = defaultdict(float)
for s, e, q, n, g in step:
    qt[q] += (e - s) / 1e3
    if want_q is not None and q != want_q:
        continue
    nm = re.sub(r"^void ", "", n)
    nm = re.sub(r"\(anonymous namespace\)::", "", nm)
    k = (q, nm.split("((")[0].split("(")[0][:70] if "<" not in nm else nm[:nm.find(">") + 1][:70], g)
    tot[k] += (e - s) / 1e3
    cnt[k] += 1
print(f"step wall {(t1 - t0) / 1e3:.1f} us; per queue {dict((q, round(v, 1)) for q, v in qt.items())}")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:top]:
    print(f"q{k[0]} {v:8.1f} us {cnt[k]:3d}x  {k[1]}  grid {k[2]}")
