"""Per-process kernel summary of a multi-process rocprofv3 kernel trace (`-o %pid%_run`): kernel
counts, mean durations and each process's busy fraction over the common window.

    python scripts/ps_trace_summary.py gpurun_out/<dir>/prof
"""
import collections
import csv
import glob
import os
import sys


def main(d):
    files = sorted(glob.glob(os.path.join(d, '*_kernel_trace.csv')))
    procs = {}
    for f in files:
        rows = [r for r in csv.DictReader(open(f)) if r['Kernel_Name'].startswith(('dqn', 'void dqn'))]
        if rows:
            procs[os.path.basename(f).split('_')[0]] = rows
    t0 = max(min(int(r['Start_Timestamp']) for r in rs) for rs in procs.values())
    t1 = min(max(int(r['End_Timestamp']) for r in rs) for rs in procs.values())
    print('common window %.1f ms' % ((t1 - t0) / 1e6))
    for pid, rs in procs.items():
        rs = [r for r in rs if t0 <= int(r['Start_Timestamp']) <= t1]
        dur = collections.defaultdict(float)
        cnt = collections.Counter()
        for r in rs:
            n = r['Kernel_Name'].replace('void ', '')[:58]
            dur[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            cnt[n] += 1
        busy = sum(dur.values())
        print('pid %s: %d kernels, kernel time %.1f%% of the window' % (pid, len(rs), 100.0 * busy * 1e3 / (t1 - t0)))
        for n, c in cnt.most_common(12):
            print('   %6d x %8.2f us  %s' % (c, dur[n] / c, n))


if __name__ == '__main__':
    main(sys.argv[1])
