#!/usr/bin/env python3
"""bench_mhap.py -- the MHAP stage on MI355X: overlaps/sec on BASELINE configs[3]
(200k synthetic raw-ONT-like reads x 15 kb, MinHash sketch + two-stage filter).

One step = one whole MHAP job over the resident read set, the jar's self search (MHAP 2.1.2
semantics, restated from its bytecode in oracle/mhap_jar.py): sketch both strands of every
read (MinHash and ordered sketches), build the MinHash index over all strands, compare every
read's forward strand against the stored strands of smaller IDs (each pair once).  With --gpus N (torchrun, one process per GPU): every rank generates 1/N
of the reads and the read store is all-gathered at setup (as bench.py does); in the timed
step each rank sketches its 1/N of the reads, the sketch rows are ALL-GATHERED over RCCL
(xGMI) -- the shared MinHash index of BASELINE configs[3] -- every rank sorts the index and
compares its own query range (ranges balanced by pair count), independent output.

Prints ONE JSON line (rank 0).  The overlapInCore headline is bench.py; this is the second
stage the north star names (src/mhap).
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

METRIC = "overlaps/sec + Gbp-vs-Gbp/sec, MHAP sketch+filter, 200k x 15 kb reads"
HBM_PEAK_GBS = 8000.0
VALU_ISSUE_PEAK_G = 256 * 4 * 2.4 / 2.0         # G wave64 VALU instructions/s: 1,024 SIMDs,
                                                # one per 2 cycles


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: the launcher's WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reads", type=int, default=200_000)
    ap.add_argument("--read-len", type=int, default=15_000)
    ap.add_argument("--coverage", type=float, default=25.0)
    ap.add_argument("--read-error", type=float, default=0.05)
    ap.add_argument("--sensitivity", default="normal")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--weighting", choices=("canu", "none"), default="canu",
                    help="canu: --repeat-weight 0.9 --repeat-idf-scale 10 with a -f table "
                         "(OverlapMhap.pm:382); none: --repeat-weight -1 (the jar's "
                         "unweighted MinHash), no table")
    ap.add_argument("--freq-kmers", type=int, default=100_000,
                    help="-f table size (16-mers sampled from the reads, graded fractions)")
    ap.add_argument("--cpu-sample-reads", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args(argv)


def workload_key(args) -> dict:
    """What the PMC figures of profiles/traffic_mhap.json were taken on (tools/pmc_mhap.py)."""
    return {"workload": "configs3", "reads": args.reads, "read_len": args.read_len,
            "coverage": args.coverage, "read_error": args.read_error,
            "sensitivity": args.sensitivity, "seed": args.seed, "weighting": args.weighting,
            "freq_kmers": args.freq_kmers}


def mhap_source_hash() -> str:
    import hashlib
    h = hashlib.sha256()
    for rel in ("canu_amd/csrc/mhap.hip", "include/canu_mhap.h"):
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def load_pmc(args, world):
    """profiles/traffic_mhap.json when taken on this workload and these sources, else None."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic_mhap.json")) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "profiles/traffic_mhap.json missing"
    meta = t.get("_method", {})
    if world != 1:
        return None, "PMC figures are single-GPU: not used at N > 1"
    if meta.get("workload") != workload_key(args):
        return None, f"PMC passes ({meta.get('tag')}) were taken on another workload"
    if meta.get("src_sha") != mhap_source_hash():
        return None, f"PMC passes ({meta.get('tag')}) were taken on other MHAP sources"
    return t, f"profiles/traffic_mhap.json ({meta.get('tag')}, same workload and sources)"


def main() -> None:
    args = parse_args()

    from canu_amd import launch
    # decide BEFORE anything touches the GPU: N ranks of this script in a child launcher
    if launch.needs_spawn(args.gpus):
        sys.exit(launch.spawn_ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    rank, world, local = launch.world_from_env(args.gpus)
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
        assert dist.get_world_size() == world, (dist.get_world_size(), world)

    from canu_amd.synth import synth_reads, random_genome
    from canu_amd.mhap import Mhap, MhapParameters
    from canu_amd.dist import gather_read_store, query_shards, read_slices, all_gather_rows

    n = args.reads
    genome_len = int(n * args.read_len / args.coverage)
    gen_kw = dict(n_reads=n, read_len=args.read_len, genome_len=genome_len,
                  error_rate=args.read_error, seed=args.seed)
    t_setup = time.time()
    genome = random_genome(np.random.default_rng(args.seed), genome_len)
    lo, hi = read_slices(n, world)[rank]
    part = synth_reads(genome=genome, read_range=(lo, hi), **gen_kw)
    dev = torch.device("cuda", local)
    if world == 1:
        bases = torch.from_numpy(part.bases).to(dev)
        lengths = part.lengths
    else:
        bases, lengths = gather_read_store(torch.from_numpy(part.bases).to(dev), part.lengths,
                                           dist, dev)
    del part
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    d_offsets = torch.from_numpy(offsets.view(np.int64)).to(dev)
    total_bases = int(lengths.sum(dtype=np.uint64))

    P = MhapParameters.sensitivity(args.sensitivity)
    freq = None
    if args.weighting == "canu":
        P.canu_weighting()
        freq = freq_table(genome, args.freq_kmers, P.k, args.seed)
    else:
        P.repeat_weight = -1.0
    m = Mhap(P, device=local)
    m.load_reads_device(1, bases.data_ptr(), d_offsets.data_ptr(), lengths)
    if freq is not None:
        m.set_kmer_frequencies(*freq)
    else:
        m.set_weighting()
    H, S = P.num_hashes, P.ordered_sketch_size
    if world > 1:                       # rows per read: both strands (canu_mhap.h)
        mh_l = torch.empty((hi - lo, 2 * H), dtype=torch.int32, device=dev)
        od_l = torch.empty((hi - lo, 2 * S), dtype=torch.int64, device=dev)
        oc_l = torch.empty((hi - lo, 2), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    q_lo, q_hi = query_shards(n, world)[rank]
    setup_s = time.time() - t_setup
    ms = {"sketch": 0.0, "index": 0.0, "candidates": 0.0, "compare": 0.0, "gather": 0.0}

    def step() -> int:
        m.sketch(lo + 1, hi)
        st = m.stats()
        ms["sketch"] += st["ms_sketch"]
        if world > 1:
            t0 = time.perf_counter()
            m.copy_sketches(lo + 1, hi - lo, mh_l.data_ptr(), od_l.data_ptr(), oc_l.data_ptr(),
                            False)
            mh = all_gather_rows(mh_l, n, dist)
            od = all_gather_rows(od_l, n, dist)
            oc = all_gather_rows(oc_l, n, dist)
            torch.cuda.synchronize()
            m.copy_sketches(1, n, mh.data_ptr(), od.data_ptr(), oc.data_ptr(), True)
            del mh, od, oc
            ms["gather"] += 1000.0 * (time.perf_counter() - t0)
        m.build_index()
        nrec = m.compare(q_lo, q_hi) if q_lo <= q_hi else 0
        st = m.stats()
        ms["index"] += st["ms_index"]
        ms["candidates"] += st["ms_candidates"]
        ms["compare"] += st["ms_compare"]
        return nrec

    for _ in range(args.warmup):
        step()
    for k in ms:
        ms[k] = 0.0
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
    st = m.stats()

    red = dev if backend == "nccl" else torch.device("cpu")
    el = torch.tensor([elapsed], dtype=torch.float64, device=red)
    nr = torch.tensor([nrec, st["candidates"]], dtype=torch.int64, device=red)
    if dist:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(nr, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    total_ovl, total_cand = int(nr[0].item()), int(nr[1].item())
    value = total_ovl * args.steps / elapsed
    gbp = total_bases / 1e9

    # Dominant kernel: the MinHash draws -- k_mh_minhash (the exact sample and the k-mers of
    # other weights) and k_mh_bitslice (the rest, 32 chains per lane in bit planes), timed
    # together live by the library's events (ms_sketch_kernel: both launches of a batch).
    # They are bound by vector-instruction issue: every distinct k-mer of both strands makes
    # w x H xorshift64 draws.  With the PMC pass of this
    # workload and these sources (profiles/traffic_mhap.json) the roofline is VALU
    # wave-instructions/s against 1,024 SIMDs x 2.4 GHz / 2 (wave64 over 2 cycles); its HBM
    # figures beside: algorithmic bytes = the sorted (key, position) pairs read once (12 B
    # per k-mer position) + the sketch rows written (4 B x H per strand).
    draws = int(st.get("sketch_draws", 0))
    nl = max(int(st.get("sketch_launches", 0)), 1)
    k_ms = st.get("ms_sketch_kernel", 0.0) / nl
    kname = "k_mh_minhash + k_mh_bitslice"
    strands = 2 * (hi - lo)
    positions = max(0, int(np.maximum(lengths[lo:hi].astype(np.int64) - P.k + 1, 0).sum())) * 2
    per_launch = (12.0 * positions + 4.0 * H * strands) / nl
    pmc, pmc_note = load_pmc(args, world)
    # the two draw kernels' per-launch figures (one launch of each per batch) added
    kp = {}
    for kk in ("k_mh_minhash", "k_mh_bitslice"):
        e = (pmc or {}).get(kk)
        if not e:
            continue
        for f in ("valu_insts", "hbm_bytes_per_launch"):
            kp[f] = kp.get(f, 0.0) + e.get(f, 0.0)
        if kk == "k_mh_bitslice":
            kp["wait_inst_any_frac"] = e.get("wait_inst_any_frac", 0.0)
    hbm = {"achieved": round(per_launch / (k_ms * 1e-3) / 1e9, 2) if k_ms > 0 else None,
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "algorithmic_bytes_per_launch": int(per_launch),
           "traffic": kp.get("hbm_bytes_per_launch")}
    if hbm["achieved"] is not None:
        hbm["frac"] = round(hbm["achieved"] / HBM_PEAK_GBS, 5)
    roof = {"kernel": kname, "launches": nl, "avg_launch_ms": round(k_ms, 3),
            "draws_per_launch": draws // nl,
            "g_draws_per_s": round(draws / nl / (k_ms * 1e-3) / 1e9, 2) if k_ms > 0 else None,
            "pmc_source": pmc_note}
    if kp and k_ms > 0:
        valu = kp["valu_insts"] / (k_ms * 1e-3) / 1e9
        pk = VALU_ISSUE_PEAK_G
        roof.update({"bound": "issue", "achieved": round(valu, 1), "peak": round(pk, 1),
                     "unit": "G VALU wave-instructions/s", "frac": round(valu / pk, 4),
                     "traffic": kp.get("hbm_bytes_per_launch"), "hbm": hbm,
                     "valu_per_draw": round(kp["valu_insts"] * 64.0 / max(draws / nl, 1.0), 2),
                     "wait_inst_any_frac": round(kp.get("wait_inst_any_frac", 0.0), 3),
                     "limiter": "vector-instruction issue: the xorshift64 draws of the "
                                "weighted MinHash (w x H per distinct k-mer and strand)"})
    else:
        roof.update({"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": hbm.get("frac"), "traffic": None,
                     "algorithmic_bytes_per_launch": int(per_launch),
                     "limiter": "VALU issue (see DESIGN.md); no PMC issue counters for this "
                                "workload and these sources, so the HBM figure is given"})

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, P, freq)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "overlaps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u8 bases, int32/u64 hash sketches", "data": "synthetic",
            "config": {"workload": "configs[3]: MHAP MinHash sketch+filter, synthetic reads, "
                                   "all-vs-all", "reads": n, "read_len": args.read_len,
                       "coverage": args.coverage, "read_error": args.read_error,
                       "sensitivity": args.sensitivity, "num_hashes": H,
                       "weighting": (f"canu (--repeat-weight 0.9 --repeat-idf-scale 10 "
                                     f"--filter-threshold {P.filter_threshold}, -f table of "
                                     f"{args.freq_kmers} 16-mers)") if freq is not None
                                    else "none (unweighted)",
                       "ordered_sketch": S, "k": P.k, "ordered_k": P.ordered_kmer_size,
                       "parallelism": f"query-shard{world}",
                       "dist_backend": backend if world > 1 else None},
            "overlaps_per_step": total_ovl, "candidates_per_step": total_cand,
            "gbp_vs_gbp_per_sec": round(gbp * gbp / 2.0 * args.steps / elapsed, 3),
            "breakdown_ms": {k: round(v / args.steps, 2) for k, v in ms.items()},
            "setup_s": round(setup_s, 1), "roofline": roof, "cpu_baseline": cpu,
            "sketch": {"kmers": int(st["sketch_kmers"]), "draws": draws,
                       "reads_used": int(st["sketched_reads"])},
            "parity": {"checked": False, "pinned": "bytecode",
                       "reason": "the GPU is bit-exact to oracle/mhap_jar.py "
                                 "(tests/test_mhap.py), the jar's bytecode restated method by "
                                 "method; no jar output exists to pin against (no JVM, no "
                                 "fixtures in the reference)"},
        }
        print(json.dumps(line), flush=True)
    m.close()
    if dist:
        dist.destroy_process_group()


def freq_table(genome, n: int, k: int, seed: int):
    """A -f table the way canu's is shaped (Meryl.pm:699-716: k-mer, fraction; both strands):
    n/2 k-mers drawn from the genome with fractions graded from the filter threshold up."""
    rng = np.random.default_rng(seed + 77)
    g = genome.tobytes().decode()
    comp = str.maketrans("ACGT", "TGCA")
    km, fr = [], []
    for j, p in enumerate(rng.integers(0, len(g) - k, size=max(n // 2, 0))):
        m = g[int(p):int(p) + k]
        f = 5e-6 * 1.3 ** (j % 24)
        km += [m, m.translate(comp)[::-1]]
        fr += [f, f]
    return km, np.array(fr, dtype=np.float64)


def cpu_baseline(args, P, freq=None) -> dict | None:
    """The numpy restatement of the jar (oracle/mhap_jar.py, one core) on a bounded sample of
    the same workload: fewer reads, same read length / error / coverage / weighting."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import mhap_jar
        from canu_amd.synth import synth_reads
    except Exception:
        return None
    ns = args.cpu_sample_reads
    gl = int(ns * args.read_len / args.coverage)
    rs = synth_reads(ns, args.read_len, gl, args.read_error, seed=args.seed + 1000)
    t0 = time.perf_counter()
    rec = mhap_jar.run(rs, P.as_oracle(), freq=freq)
    secs = time.perf_counter() - t0
    return {"value": round(len(rec) / secs, 2), "unit": "overlaps/s", "cores": 1,
            "kind": "port",
            "sample": f"{ns} reads x {args.read_len} bp at {args.coverage:.0f}x (genome {gl} bp), "
                      f"numpy restatement {secs:.1f}s, {len(rec)} overlaps"}


if __name__ == "__main__":
    main()
