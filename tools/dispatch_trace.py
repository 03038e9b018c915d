#!/usr/bin/env python3
"""Per-dispatch kernel durations (us) from a rocprofv3 --kernel-trace run
(sqlite results .db); with a name filter, the last N matching dispatches."""
import glob
import os
import sqlite3
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
last = int(sys.argv[3]) if len(sys.argv) > 3 else 60
dbs = [src] if os.path.isfile(src) else glob.glob(os.path.join(src, "**", "*.db"), recursive=True)
for p in dbs:
    db = sqlite3.connect(p)
    rows = list(db.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                           "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"))
    sel = [(n.split("(")[0].split("::")[-1], s, e) for n, s, e in rows if pat in n]
    t0 = sel[-last][1] if len(sel) >= last else (sel[0][1] if sel else 0)
    for n, s, e in sel[-last:]:
        print("%-28s start %9.1f dur %8.1f" % (n[:28], (s - t0) / 1e3, (e - s) / 1e3))
