"""Per-kernel duration stats from a rocprofv3 results database (rocpd sqlite, the default output
format): name, calls, avg / min / max us, share.  Usage: rocpd_stats.py <run_results.db> [top]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 16
names = {r[0]: r[1] for r in db.execute("select id, display_name from rocpd_info_kernel_symbol")}
d = collections.defaultdict(list)
for kid, s, e in db.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
    d[names.get(kid, str(kid))].append((e - s) / 1e3)
tot = sum(sum(v) for v in d.values())
print("| kernel | calls | avg µs | min µs | max µs | share % |\n|---|---|---|---|---|---|")
for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print("| `%s` | %d | %.1f | %.1f | %.1f | %.1f |" % (n[:90], len(v), sum(v) / len(v), min(v), max(v), 100 * sum(v) / tot))
