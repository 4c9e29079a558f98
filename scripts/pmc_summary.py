"""Summarise rocprofv3 --pmc counter CSVs (scripts/profile_counters.sh) per kernel:
MFMA FLOPs per type (bf16 / fp16 / fp32: SQ_INSTS_VALU_MFMA_MOPS_* count 512 FLOPs each) and busy %,
LDS bank-conflict rate, HBM bytes, achieved rates."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))   # kernel -> counter -> sum
calls = collections.defaultdict(set)
dur = collections.defaultdict(float)
for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(path)):
        k = r.get('Kernel_Name', '?')
        vals[k][r['Counter_Name']] += float(r['Counter_Value'])
        calls[k].add((path, r.get('Dispatch_Id', r.get('Correlation_Id', ''))))
for path in glob.glob(os.path.join(root, '**', '*kernel_trace.csv'), recursive=True):
    if 'pass1' not in path:
        continue
    for r in csv.DictReader(open(path)):
        dur[r['Kernel_Name']] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9


def short(k):
    k = k.replace('void ', '')
    return (k[:70] + '...') if len(k) > 73 else k


print('| kernel | dispatches | time ms | MFMA GFLOP bf16 / fp16 / fp32 | MFMA TFLOP/s | MFMA busy % of kernel '
      '| LDS conflict % | HBM read MB | HBM write MB | HBM GB/s |')
print('|---|---|---|---|---|---|---|---|---|---|')
rows = sorted(vals.items(), key=lambda kv: -dur.get(kv[0], 0.0))
for k, c in rows:
    if not k.startswith(('dqn', 'void dqn', '_ZN3dqn')):
        continue
    n = len({d for p, d in calls[k] if 'pass1' in p}) or 1
    t = dur.get(k, 0.0)
    fb, fh, ff = (c.get('SQ_INSTS_VALU_MFMA_MOPS_' + x, 0.0) * 512 for x in ('BF16', 'F16', 'F32'))
    fl = fb + fh + ff
    busy = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0)
    gui = c.get('GRBM_GUI_ACTIVE', 0.0)
    mfma_pct = 100.0 * busy / (gui * 4 * 256) if gui else 0.0       # 4 SIMDs x 256 CUs
    lds = c.get('SQ_LDS_IDX_ACTIVE', 0.0)
    conf = 100.0 * c.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds if lds else 0.0
    rd, wr = c.get('FETCH_SIZE', 0.0) / 1024, c.get('WRITE_SIZE', 0.0) / 1024     # KB -> MB
    bw = (rd + wr) / 1024 / t if t else 0.0
    print('| %s | %d | %.3f | %.3f / %.3f / %.3f | %.2f | %.1f | %.1f | %.2f | %.2f | %.0f |' % (
        short(k), n, t * 1e3, fb / 1e9, fh / 1e9, ff / 1e9, fl / t / 1e12 if t else 0.0, mfma_pct, conf, rd, wr, bw))
