"""Summarise a rocprofv3 SQLite result (kernel name, calls, total/avg us)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
q = (f"select {name}, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels "
     f"group by {name} order by sum(end-start) desc limit {int(sys.argv[2]) if len(sys.argv) > 2 else 30}")
for nm, c, tot, avg in db.execute(q):
    print(f"{tot:12.1f} us {c:7d} x {avg:9.2f} us  {nm[:110]}")
