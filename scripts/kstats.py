"""Summarise a rocprofv3 kernel-trace CSV: per kernel (and grid) average durations."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[(r['Kernel_Name'][:80], r['Grid_Size_X'], r['Grid_Size_Y'])].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print('%-80s %7s %3s %6d %8.2fus %5.1f%%' % (k[0], k[1], k[2], len(v), sum(v) / len(v) / 1e3, 100 * sum(v) / tot))
