"""Gap analysis of a three-stream kernel trace (rocprofv3 --kernel-trace csv): over the timed
steady state, the share of wall time with a scan kernel running, and what runs (or nothing)
while none does.  Usage: timeline6.py run_kernel_trace.csv
The window is the densest run of 40 consecutive launches of the scan kernel named by the optional
second argument (the bench's timed three-stream loop; its p50 loop after it runs one batch at a
time with a host sync per batch, which an earlier version of this script took by mistake)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    n = r['Kernel_Name']
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    short = n.split('(')[0].replace('void ', '').replace('vdb::', '')
    ev.append((s, e, short, int(r.get('Stream_Id', 0) or 0)))
ev.sort()
pat = sys.argv[2] if len(sys.argv) > 2 else 'scan8'
scans = [x for x in ev if pat in x[2] and 'exact' not in x[2]]
# steady state: the densest 40 consecutive scans (the timed loop)
j = min(range(len(scans) - 39), key=lambda i: scans[i + 39][1] - scans[i][0])
scans = scans[j:j + 40]
t0, t1 = scans[0][0], scans[-1][1]
win = [x for x in ev if x[1] > t0 and x[0] < t1]
# sweep over time points
pts = sorted({t0, t1} | {max(t0, x[0]) for x in win} | {min(t1, x[1]) for x in win})
no_scan = 0
alone = defaultdict(float)
for a, b in zip(pts, pts[1:]):
    if b <= a:
        continue
    mid = (a + b) / 2
    act = [x[2] for x in win if x[0] <= mid < x[1]]
    if not any('scan8' in k and 'exact' not in k for k in act):
        no_scan += b - a
        key = ' + '.join(sorted(set(k[:28] for k in act))) or '(idle)'
        alone[key] += b - a
tot = t1 - t0
print('window %.1f us over %d scans: %.1f us per scan-step; scan running %.1f%%' % (tot / 1e3, len(scans), tot / 1e3 / len(scans), 100 * (1 - no_scan / tot)))
print('without a scan, per step (us):')
for k, v in sorted(alone.items(), key=lambda kv: -kv[1])[:12]:
    print('  %7.2f  %s' % (v / 1e3 / len(scans), k))
dur = defaultdict(list)
for x in win:
    dur[x[2][:40]].append(x[1] - x[0])
print('mean durations in the window (us):')
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print('  %7.1f x%3d  %s' % (sum(v) / len(v) / 1e3, len(v), k))
