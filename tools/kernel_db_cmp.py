#!/usr/bin/env python3
"""Average kernel durations from rocprofv3 --kernel-trace SQLite outputs, side by side.
    python tools/kernel_db_cmp.py PATTERN run_a/run_results.db run_b/run_results.db ..."""
import sqlite3
import sys

pat, dbs = sys.argv[1], sys.argv[2:]
rows = {}
for i, p in enumerate(dbs):
    db = sqlite3.connect(p)
    q = "select name, count(*), avg(end - start) / 1e3 from kernels where name like ? group by name"
    for name, c, avg in db.execute(q, (f"%{pat}%",)):
        rows.setdefault(name.split("(")[0][:48], {})[i] = (c, avg)
print("kernel".ljust(48), *[f"{p.split('/')[-2]:>16}" for p in dbs])
for name, d in sorted(rows.items()):
    print(name.ljust(48), *[f"{d[i][1]:>10.1f} us x{d[i][0]:<3}" if i in d else " " * 16 for i in range(len(dbs))])
