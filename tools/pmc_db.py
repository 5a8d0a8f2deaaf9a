#!/usr/bin/env python3
"""Per-kernel PMC counter sums from rocprofv3 sqlite outputs (gpurun_out/<dir>/*.db).
    python tools/pmc_db.py gpurun_out/pmcA_1 [gpurun_out/pmcA_2 ...]"""
import collections
import glob
import sqlite3
import sys

for d in sys.argv[1:]:
    for db in glob.glob(d + "/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = """select ks.kernel_name, p.name, sum(e.value), count(distinct kd.id)
               from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id
               join rocpd_kernel_dispatch kd on e.event_id = kd.event_id
               join rocpd_info_kernel_symbol ks on kd.kernel_id = ks.id
               group by ks.kernel_name, p.name"""
        try:
            rows = c.execute(q).fetchall()
        except sqlite3.Error as ex:
            print(db, ex)
            continue
        agg = collections.defaultdict(dict)
        for k, n, v, cnt in rows:
            agg[k.split("(")[0]][n] = (v, cnt)
        for k in sorted(agg):
            print(k, {n: f"{v:.4g}" for n, (v, _) in sorted(agg[k].items())})
