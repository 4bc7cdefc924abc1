"""Per-kernel totals from a rocprofv3 rocpd database (--kernel-trace): name, calls, total ms, avg ms."""
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end-start)/1e6, avg(end-start)/1e6 from kernels group by name order by 3 desc").fetchall()
for r in rows:
    print("%-44s %6d %10.3f %9.4f" % (r[0][:44], r[1], r[2], r[3]))
