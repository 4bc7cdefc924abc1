#!/usr/bin/env python3
"""Kernel time summary from a rocprofv3 rocpd database (run_results.db): name, calls, total and
average ms, sorted by total.  Usage: tools/kt_db.py gpurun_out/devkt/run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end - start), avg(end - start) from kernels group by name "
                 "order by sum(end - start) desc").fetchall()
for name, n, tot, avg in rows:
    print("%-40s %5d %12.3f ms %10.3f ms" % (name.split("(")[0][:40], n, tot / 1e6, avg / 1e6))
