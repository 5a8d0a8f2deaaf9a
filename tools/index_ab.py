"""Index-build A/B: time build_hash_index over the bench's read set for one library build
(CANU_OVL_LIB selects it) and print the per-build ms plus a result fingerprint (the seed
hits and overlaps of a small query range) so variants can be checked against each other.

usage: CANU_OVL_LIB=canu_amd/lib/ab_x.so python tools/index_ab.py [--reads N] [--reps R]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000)
    ap.add_argument("--read-len", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--finds", type=int, default=1, help="full searches (median extend ms)")
    args = ap.parse_args()
    import torch
    from canu_amd.synth import synth_reads, random_genome
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore

    n = args.reads
    genome_len = int(n * args.read_len / 25.0)
    genome = random_genome(np.random.default_rng(1), genome_len)
    part = synth_reads(genome=genome, read_range=(0, n), n_reads=n, read_len=args.read_len,
                       genome_len=genome_len, error_rate=0.015, seed=1)
    dev = torch.device("cuda", 0)
    bases = torch.from_numpy(part.bases).to(dev)
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(part.lengths[:-1], dtype=np.uint64)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(dev)
    P = OicParameters(Kmer_Len=22, maxErate=float(np.float32(0.06)), Min_Olap_Len=500).finalize()
    oic = OverlapInCore(P, device=0)
    oic.load_reads_device(1, bases.data_ptr(), d_off.data_ptr(), part.lengths)
    torch.cuda.synchronize()
    ms = []
    for _ in range(args.reps + 1):
        t0 = time.perf_counter()
        oic.build_hash_index(1, n)
        torch.cuda.synchronize()
        ms.append(1000.0 * (time.perf_counter() - t0))
        ms[-1] = (ms[-1], oic.stats()["ms_index"])
    if args.finds == 0:           # timing only (phase-cut builds leave no usable index)
        wall = sorted(x[0] for x in ms[1:])
        ev = sorted(x[1] for x in ms[1:])
        print(f"{os.path.basename(os.environ.get('CANU_OVL_LIB', 'libcanu_ovl.so'))}: index ms "
              f"wall min {wall[0]:.2f} med {wall[len(wall) // 2]:.2f}, events med "
              f"{ev[len(ev) // 2]:.2f}", flush=True)
        return
    ext, seed = [], []
    for _ in range(args.finds):
        novl = oic.find_overlaps(1, n)
        st = oic.stats()
        ext.append(st.get("ms_extend", 0.0))
        seed.append(st.get("ms_seed", 0.0))
    st["ms_extend"] = sorted(ext)[len(ext) // 2]
    st["ms_seed"] = sorted(seed)[len(seed) // 2]
    import zlib
    crc = zlib.crc32(np.ascontiguousarray(oic.fetch()).tobytes())
    wall = sorted(x[0] for x in ms[1:])
    ev = sorted(x[1] for x in ms[1:])
    print(f"{os.path.basename(os.environ.get('CANU_OVL_LIB', 'libcanu_ovl.so'))}: index ms "
          f"wall min {wall[0]:.2f} med {wall[len(wall) // 2]:.2f}, events med "
          f"{ev[len(ev) // 2]:.2f} | fingerprint overlaps {novl} "
          f"crc {crc:08x} seed_hits {st.get('seed_hits')} | probe ms {st.get('ms_probe_kernel'):.2f} seed ms {st.get('ms_seed'):.2f} extend ms "
          f"{st.get('ms_extend', 0):.1f}", flush=True)


if __name__ == "__main__":
    main()
