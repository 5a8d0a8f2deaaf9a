#!/usr/bin/env python3
"""bench.py -- overlapInCore on MI355X: overlaps/sec on 50k x 10 kb synthetic ONT reads.

One step = one full overlapInCore job over the resident read set: Build_Hash_Index over
all reads (-h 1-N) and Find_Overlaps for every query read in both orientations (-r), with
seed extension and ovOverlap output (BASELINE configs[2]).  Reads are generated
synthetically (no datasets here), packed into HBM before the timed region; records stay in
HBM.  With --gpus N (torchrun, one process per GPU) every rank generates 1/N of the reads,
the packed read store is all-gathered over RCCL, every rank builds the index and searches
its own query range (ranges balanced by pair count), independent per-shard output.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "overlaps/sec + Gbp-vs-Gbp/sec, 50k×10kb ONT reads, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PROBE_BYTES_PER_WINDOW = 24.25  # k_probe: 16-B table entry + 8-B record + the 2-bit query
RAND_LOOKUP_GPS = 39.2          # G random 16-B loads/s, 16 GiB table (tools/rand_ceiling.hip)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=50_000)
    ap.add_argument("--read-len", type=int, default=10_000)
    ap.add_argument("--coverage", type=float, default=25.0)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--maxerate", type=float, default=0.06)
    ap.add_argument("--minlength", type=int, default=500)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-sample-reads", type=int, default=1000)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-seed-only", action="store_true",
                    help="skip the configs[1] seed-hit figure (profiling passes)")
    ap.add_argument("--no-shard-timing", action="store_true",
                    help="skip the per-shard timing (1 GPU: each of the 8 query shards in turn)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (1-GPU box): CANU_DEVICE pins every rank to one device,
    # CANU_DIST_BACKEND=gloo replaces RCCL; the driver's multi-GPU runs use neither
    local = int(os.environ.get("CANU_DEVICE", local))
    backend = os.environ.get("CANU_DIST_BACKEND", "nccl")

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from canu_amd.synth import synth_reads, random_genome
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    from canu_amd.dist import gather_read_store, query_shards

    n = args.reads
    genome_len = int(n * args.read_len / args.coverage)
    gen_kw = dict(n_reads=n, read_len=args.read_len, genome_len=genome_len,
                  error_rate=args.read_error, seed=args.seed)

    # ---- setup: each rank generates its slice, then the read store is all-gathered ----
    t_setup = time.time()
    genome = random_genome(np.random.default_rng(args.seed), genome_len)
    lo = n * rank // world
    hi = n * (rank + 1) // world
    part = synth_reads(genome=genome, read_range=(lo, hi), **gen_kw)
    dev = torch.device("cuda", local)
    if world == 1:
        bases = torch.from_numpy(part.bases).to(dev)
        lengths = part.lengths
    else:
        bases, lengths = gather_read_store(torch.from_numpy(part.bases).to(dev), part.lengths,
                                           dist, dev)          # RCCL over xGMI
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    d_offsets = torch.from_numpy(offsets.view(np.int64)).to(dev)
    total_bases = int(lengths.sum(dtype=np.uint64))

    P = OicParameters(Kmer_Len=args.k, maxErate=float(np.float32(args.maxerate)),
                      Min_Olap_Len=args.minlength).finalize()
    oic = OverlapInCore(P, device=local)
    oic.load_reads_device(1, bases.data_ptr(), d_offsets.data_ptr(), lengths)
    torch.cuda.synchronize()
    shards = query_shards(n, world)
    q_lo, q_hi = shards[rank]
    setup_s = time.time() - t_setup

    # each rank indexes reads q_lo..n only: its queries' targets all have larger IDs
    # (Find_Overlaps.C:328), so records and counters equal the whole index's
    def step() -> int:
        oic.build_hash_index(q_lo, n)
        return oic.find_overlaps(q_lo, q_hi)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nrec = 0
    for _ in range(args.steps):
        nrec = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = oic.stats()

    red = dev if backend == "nccl" else torch.device("cpu")
    el = torch.tensor([elapsed], dtype=torch.float64, device=red)
    nr = torch.tensor([nrec], dtype=torch.int64, device=red)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(nr, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_ovl = int(nr.item())
    value = total_ovl * args.steps / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    gbp = total_bases / 1e9
    gbp_vs_gbp = gbp * gbp / 2.0 * args.steps / elapsed    # all-vs-all, each pair once

    traffic = load_traffic()
    # Dominant kernel: k_extend (the banded edit-distance extension).  Its algorithmic HBM
    # bytes per pair are the two packed strands it stages (2 bits/base + guard word each),
    # the pair's seed-match nodes (16 B each, read once: the Add_Match lists, not the seed
    # hits they merge -- rounds before r02v counted 16 B per hit, ~7x the bytes) and its
    # output records (24 B each); per launch
    # = the step's bytes / the step's launches, over the launches' average duration (HIP
    # events on the library's stream).
    avg_len = total_bases / max(n, 1)
    strand = 8.0 * (np.ceil(avg_len / 32.0) + 1.0)
    ext_bytes = st["pairs"] * 2 * strand + st["seed_nodes"] * 16 + st["total_overlaps"] * 24
    roof = None
    n_ext = max(int(st.get("extend_launches", 0)), 1)
    if st["ms_extend"] > 0:
        per_launch = ext_bytes / n_ext
        avg_ms = st["ms_extend"] / n_ext
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": _traffic(traffic, "k_extend"), "kernel": "k_extend",
                "limiter": "instruction issue of the greedy O(ND) rows: the per-row scalar "
                           "control (SALU, shared by a CU's 4 SIMDs) first, then integer VALU; "
                           "no MFMA shape, HBM far from busy",
                "issue": traffic.get("k_extend", {}).get("issue"),
                "algorithmic_bytes_per_launch": int(per_launch), "launches": n_ext,
                "avg_launch_ms": round(avg_ms, 3)}
    # The north star's roofline target: the hash-probe kernel (one 16-B table entry and one
    # 8-B probe record per query window, plus the 2-bit query).
    probe_roof = None
    n_pr = max(int(st.get("probe_launches", 0)), 1)
    if st["ms_probe_kernel"] > 0:
        per_launch = st["probe_bytes"] / n_pr
        avg_ms = st["ms_probe_kernel"] / n_pr
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        probe_roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                      "traffic": _traffic(traffic, "k_probe"), "kernel": "k_probe",
                      "algorithmic_bytes_per_launch": int(per_launch), "launches": n_pr,
                      "avg_launch_ms": round(avg_ms, 3)}
        # the same launch against the roofline in the bytes it actually moves (PMC traffic
        # per launch over this run's launch time): one 64-B sector per 16-B slot probed
        tb = probe_roof["traffic"]
        if tb:
            probe_roof["traffic_gbs"] = round(tb / (avg_ms * 1e-3) / 1e9, 1)
            probe_roof["traffic_frac"] = round(probe_roof["traffic_gbs"] / HBM_PEAK_GBS, 4)
        # the achievable bound of a one-random-lookup-per-window probe: independent random
        # 16-B loads over a 16 GiB table (this workload's) sustain 39.2 G/s at any depth of
        # memory-level parallelism (tools/rand_ceiling.hip, profiles/r02w_rand_ceiling.log)
        wps = achieved * 1e9 / PROBE_BYTES_PER_WINDOW
        probe_roof["random_lookup_ceiling"] = {
            "windows_per_s": round(wps / 1e9, 2), "ceiling_gloads_per_s": RAND_LOOKUP_GPS,
            "frac_of_ceiling": round(wps / 1e9 / RAND_LOOKUP_GPS, 3),
            "source": "profiles/r02w_rand_ceiling.log (16 GiB table)"}

    # BASELINE configs[1] on the same read set: the hash index + seed-hit kernels alone (the
    # Add_Ref hit list of every query, both orientations, written to HBM, not copied out);
    # a 1-GPU figure (at N > 1 a rank would report only its own shard's hits)
    seed_only = None
    if world == 1 and not args.no_seed_only:
        oic.build_hash_index(q_lo, n)
        n_hits = oic.seed_hits(q_lo, q_hi, fetch=False)
        st1 = oic.stats()
        seed_only = {"workload": "configs[1]: hash index + seed-hit list, same reads",
                     "seed_hits": n_hits, "ms_index": round(st1["ms_index"], 2),
                     "ms_seed_hits": round(st1["ms_seed_hits"], 2),
                     "seed_hits_per_s": round(n_hits / ((st1["ms_index"] + st1["ms_seed_hits"])
                                                        * 1e-3), 1)}

    # Multi-GPU evidence from one GPU: the 8-way query shards (dist.query_shards) one after
    # another, each with its own index build, as each rank of an 8-GPU job runs them
    shard = None
    if world == 1 and not args.no_shard_timing:
        shard_ms = []
        for lo8, hi8 in query_shards(n, 8):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            oic.build_hash_index(lo8, n)
            oic.find_overlaps(lo8, hi8)
            torch.cuda.synchronize()
            shard_ms.append(round(1000.0 * (time.perf_counter() - t1), 1))
        shard = {"shards": 8, "shard_ms": shard_ms,
                 "projected_speedup_8": round(sum(shard_ms) / max(shard_ms), 2),
                 "projected_vs_1gpu_step": round(ms_step / max(shard_ms), 2),
                 "note": "the 8 ranks' jobs (index over the shard's lo..n, then its queries) "
                         "timed in turn on one GPU; projected_speedup_8 = sum / max, "
                         "projected_vs_1gpu_step = this run's 1-GPU step / the slowest rank; "
                         "the driver's 8-GPU run measures the real curve"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "overlaps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u8/2-bit bases, int32 edit rows", "data": "synthetic",
            "config": {"workload": "configs[2]: 50k synthetic ONT reads x 10 kb, full "
                                   "overlapInCore (seed + banded extend), all-vs-all",
                       "reads": n, "read_len": args.read_len, "coverage": args.coverage,
                       "read_error": args.read_error, "k": args.k,
                       "maxerate": P.maxErate, "minlength": args.minlength,
                       "parallelism": f"query-shard{world}"},
            "overlaps_per_step": total_ovl,
            "gbp_vs_gbp_per_sec": round(gbp_vs_gbp, 4),
            "breakdown_ms": {"index": round(st["ms_index"], 2), "seed": round(st["ms_seed"], 2),
                             "extend": round(st["ms_extend"], 2)},
            "seed_hits": st["seed_hits"], "seed_nodes": st["seed_nodes"], "pairs": st["pairs"],
            "setup_s": round(setup_s, 1),
            "roofline": roof,
            "probe_roofline": probe_roof,
            "seed_only": seed_only,
            "shard_timing": shard,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    oic.close()
    if dist:
        dist.destroy_process_group()


def _traffic(t: dict, k: str):
    """HBM bytes per launch of kernel k from the committed PMC passes (same unit as
    algorithmic_bytes_per_launch), or None."""
    v = t.get(k)
    return None if v is None else v.get("hbm_bytes_per_launch")


def load_traffic() -> dict:
    """Per-kernel HBM traffic of one default bench step from the committed rocprofv3 PMC
    passes (profiles/traffic.json, tools/pmc_traffic.py): (r x FETCH_SIZE + WRITE_SIZE) KiB
    with r the read correction calibrated per access pattern (profiles/calib_traffic.json:
    2 for coalesced streams, 1 for k_probe's random 16-B table loads).  Empty when absent."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def cpu_baseline(args) -> dict | None:
    """The reference overlapInCore (oracle/_ref/oic_ref, built from its sources) on a
    bounded sample of the same workload: fewer reads, same read length / error / coverage,
    with canu's production hash settings -- utgOvlHashBits 23, utgOvlHashLoad 0.75
    (Defaults.pm:687-688) -- and the sample split into three hash batches (--hashstrings).
    Threads: the GPU box's CPU share (16 per GPU), not os.cpu_count(), which there reports
    the whole host; a per-core figure is given for scaling to other hosts."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle
        from canu_amd.synth import synth_reads
    except Exception:
        return None
    if not oracle.reference_available():
        return None
    ns = args.cpu_sample_reads
    gl = int(ns * args.read_len / args.coverage)
    rs = synth_reads(ns, args.read_len, gl, args.read_error, seed=args.seed + 1000)
    p = oracle.default_params(kmer_len=args.k, max_erate=args.maxerate,
                              min_olap_len=args.minlength)
    threads = min(args.cpu_threads, os.cpu_count() or 1)
    # three hash batches by --hashstrings (a --hashdatalen below the range's bases trips
    # the reference's assert at Build_Hash_Index.C:523)
    strings = (rs.nreads + 2) // 3
    datalen = rs.total_bases() + rs.nreads + 1
    rec, secs, wall = oracle.run_reference(
        rs, p, threads=threads, hash_bits=23, with_time=True,
        batching={"hashstrings": strings, "hashdatalen": datalen, "hashload": 0.75})
    v = len(rec) / secs
    return {"value": round(v, 1), "unit": "overlaps/s", "cores": threads,
            "kind": "reference", "per_core": round(v / threads, 1),
            "host_cpus": os.cpu_count(),
            "sample": f"{ns} reads x {args.read_len} bp at {args.coverage:.0f}x "
                      f"(genome {gl} bp), --hashbits 23 --hashload 0.75 --hashstrings {strings} "
                      f"(3 hash batches), reference OverlapDriver() wall {secs:.2f}s incl. its "
                      f".ovb writing, {len(rec)} overlaps"}


if __name__ == "__main__":
    main()
