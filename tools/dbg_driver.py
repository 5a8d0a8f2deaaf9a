#!/usr/bin/env python3
"""One test_driver.py case through ovl_overlap_driver under OVL_SQ = 0 / 1 / 2 (and, with
--env, any other knob): record counts, -s counters and hash batches per mode, beside the
oracle's.  usage: python tools/dbg_driver.py [case]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from canu_amd.synth import synth_reads  # noqa: E402
from test_driver import CASES, _driver_kw, _params  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "table_load"
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2"]
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    kw, batch, threads, rr = CASES[case]
    rs = synth_reads(**kw)
    P = _params()
    want, wst, batches = oracle.run_oracle_driver(
        rs, P, ref_range=rr or (1, oracle.UINT32_MAX), threads=threads, with_stats=True,
        **_driver_kw(batch))
    print(f"oracle: {want.shape[0]} records, {len(batches)} batches {batches[:4]}..., "
          f"total {wst['total_overlaps']} hits_with {wst['kmer_hits_with_olap']}", flush=True)
    d = _driver_kw(batch)
    for m in modes:
        os.environ["OVL_SQ"] = m.rstrip("c")
        if m.endswith("c"):
            os.environ["OVL_SQ_CHECK"] = "1"
        else:
            os.environ.pop("OVL_SQ_CHECK", None)
        O = OicParameters(Kmer_Len=22, maxErate=P["max_erate"], Min_Olap_Len=500,
                          Max_Hash_Strings=d["hashstrings"], Max_Hash_Data_Len=d["hashdatalen"],
                          Hash_Mask_Bits=d["hashbits"], Max_Hash_Load=d["hashload"],
                          Num_PThreads=threads).finalize()
        if rr:
            O.bgnRefID, O.endRefID = rr
        oic = OverlapInCore(O, device=0)
        got = oic.run_driver(rs)
        st = oic.stats()
        oic.close()
        same = got.shape == want.shape and np.array_equal(got, want)
        a_got = set(np.unique(got["a"]).tolist()) if got.shape[0] else set()
        a_want = set(np.unique(want["a"]).tolist())
        print(f"OVL_SQ={m}: {got.shape[0]} records, same={same}, batches {st['hash_batches']}, "
              f"total {st['total_overlaps']} hits_with {st['kmer_hits_with_olap']} "
              f"seed_hits {st['seed_hits']} pairs {st['pairs']} probe_launches "
              f"{st.get('probe_launches')} | a-reads missing {sorted(a_want - a_got)[:20]}",
              flush=True)


if __name__ == "__main__":
    main()
