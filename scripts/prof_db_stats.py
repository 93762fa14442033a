"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd sqlite): per kernel the
number of dispatches, total and average duration (ms) -- the --stats summary, as CSV."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = 'kernel_name' if 'kernel_name' in cols else 'name'
rows = c.execute("select %s, count(*), sum(end - start) from kernels group by %s order by sum(end - start) desc" % (name, name)).fetchall()
print('kernel,calls,total_ms,avg_ms')
for n, k, t in rows:
    short = n.split('(')[0][:90]
    print('%s,%d,%.3f,%.4f' % (short.replace(',', ';'), k, t / 1e6, t / 1e6 / k))
