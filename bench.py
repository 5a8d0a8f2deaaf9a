#!/usr/bin/env python3
"""bench.py -- overlapInCore on MI355X: overlaps/sec on 50k x 10 kb synthetic ONT reads.

One step = one full overlapInCore job over the resident read set: Build_Hash_Index over
all reads (-h 1-N) and Find_Overlaps for every query read in both orientations (-r), with
seed extension and ovOverlap output (BASELINE configs[2]).  Reads are generated
synthetically (no datasets here), packed into HBM before the timed region; records stay in
HBM.  After the timed region the last step's records are fetched and compared with the
reference's own output for the same reads (tests/golden/bench50k.json: count, SHA-256 of
the sorted records, an additive multiset hash, the -s counters) -> "parity".

--gpus N: one process per GPU.  Under a launcher (torch.distributed.run sets WORLD_SIZE)
the world must have N ranks; without one, N > 1 starts N ranks itself (canu_amd/launch.py).
Every rank generates 1/N of the reads, the packed read store is all-gathered over RCCL,
every rank indexes its query shard's reads lo..n and searches its own query range; the
shards' outputs are independent (no data-path collective).

--workload configs4-rank: one rank's job of BASELINE configs[4]'s 8-GPU plan at 1/8 scale
(500k x 12 kb +-20 % at 15x; the plan of canu_amd/dist.hash_block_jobs; one
`-h lo-hi -r 1-hi` OverlapDriver job with canu's --hashbits 23 --hashload 0.75 batches).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "overlaps/sec + Gbp-vs-Gbp/sec, 50k×10kb ONT reads, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
CLOCK_GHZ = 2.4                # MI355X_MICROARCH.md: max clock
N_CU, N_SIMD = 256, 1024
PROBE_BYTES_PER_WINDOW = 24.25  # k_probe: 16-B table entry + 8-B record + the 2-bit query
GOLDEN = os.path.join(ROOT, "tests", "golden", "bench50k.json")
# PMC figures per workload (tools/pmc_traffic.py): used only for a run of the same workload
# on the same kernel sources
TRAFFIC_FILES = {"configs2": "traffic.json", "configs4-rank": "traffic_configs4.json"}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default: the launcher's WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("configs2", "configs4-rank"), default="configs2")
    ap.add_argument("--reads", type=int, default=None)
    ap.add_argument("--read-len", type=int, default=None)
    ap.add_argument("--coverage", type=float, default=None)
    ap.add_argument("--read-error", type=float, default=0.015)
    ap.add_argument("--k", type=int, default=22)
    ap.add_argument("--maxerate", type=float, default=0.06)
    ap.add_argument("--minlength", type=int, default=500)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--rank-job", type=int, default=0,
                    help="configs4-rank on one GPU: which of the 8 ranks' jobs to time")
    ap.add_argument("--cpu-sample-reads", type=int, default=1500)
    ap.add_argument("--cpu-batches", type=int, default=5)
    ap.add_argument("--cpu-max-threads", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the record digest check")
    ap.add_argument("--no-seed-only", action="store_true",
                    help="skip the configs[1] seed-hit figure (profiling passes)")
    ap.add_argument("--no-shard-timing", action="store_true",
                    help="skip the per-shard timing (1 GPU: each of the 8 query shards in turn)")
    ap.add_argument("--ovb-out", default=None,
                    help="after the timed region, write the last job's records as the job's "
                         ".ovb + .counts (+ the -s stats) into this directory and time it "
                         "(configs[4]'s per-rank output, overlapInCore.C:197)")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side lines (configs[4] rank job, MHAP configs[3]) that the "
                         "default 1-GPU run adds after the headline")
    a = ap.parse_args(argv)
    c4 = a.workload == "configs4-rank"
    if a.reads is None:
        a.reads = 500_000 if c4 else 50_000
    if a.read_len is None:
        a.read_len = 12_000 if c4 else 10_000
    if a.coverage is None:
        a.coverage = 15.0 if c4 else 25.0
    if a.seed is None:
        a.seed = 5 if c4 else 1
    return a


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
    dev = torch.device("cuda", local)
    job = (Configs4Rank if args.workload == "configs4-rank" else Configs2)(args, rank, world, dev)
    # the read set is generated on the host before anything touches the GPU: its generator
    # may fork a worker pool, which must not happen after GPU initialisation
    t_setup = time.time()
    job.generate()
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == world, (dist.get_world_size(), world)
    job.dist = dist
    from canu_amd.overlap_in_core import OicParameters, OverlapInCore
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    def reduce(v, op, dtype):
        t = torch.tensor([v], dtype=dtype, device=red_dev)
        if dist:
            dist.all_reduce(t, op=op)
        return t.item()

    job.setup(OicParameters, OverlapInCore)
    setup_s = time.time() - t_setup
    # what the setup leaves on the device before the first job plans its buffers from free
    # HBM: torch should hold nothing (the staged bases are freed), the library its read store
    free_b, tot_b = torch.cuda.mem_get_info(dev)
    setup_hbm = {"device_free_gb": round(free_b / 1e9, 2), "device_total_gb": round(tot_b / 1e9, 2),
                 "torch_reserved_gb": round(torch.cuda.memory_reserved(dev) / 1e9, 3)}
    oic = job.oic

    for _ in range(args.warmup):
        job.step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nrec = 0
    for _ in range(args.steps):
        nrec = job.step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    st = oic.stats()

    SUM, MAX = (dist.ReduceOp.SUM, dist.ReduceOp.MAX) if dist else (None, None)
    elapsed = float(reduce(elapsed, MAX, torch.float64))
    total_ovl = int(reduce(nrec, SUM, torch.int64))
    value = total_ovl * args.steps / elapsed
    ms_step = 1000.0 * elapsed / args.steps
    gbp = job.total_bases / 1e9
    gbp_vs_gbp = gbp * gbp / 2.0 * args.steps / elapsed    # all-vs-all, each pair once

    # ---- parity of the last step's records against the reference's digest ------------
    parity = None
    if not args.no_parity:
        parity = job.parity(st, reduce, SUM, torch)

    roof, probe_roof, traffic_note = rooflines(args, job, st, world)
    ovb = job.write_output(args.ovb_out) if args.ovb_out else None

    seed_only = job.seed_only() if world == 1 and not args.no_seed_only else None
    shard = job.shard_timing(ms_step) if world == 1 and not args.no_shard_timing else None
    xgmi = None
    # over RCCL; on the one-GPU rehearsal (CANU_DEVICE, gloo) too, for the path's logic
    if world > 1 and (backend == "nccl" or "CANU_DEVICE" in os.environ):
        try:
            xgmi = job.index_allgather_timing(torch)
        except Exception as e:          # a side measurement: never lose the bench line to it
            xgmi = {"error": f"{type(e).__name__}: {e}"[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "configs2":
        cpu = cpu_baseline(args)

    side = None
    if rank == 0 and world == 1 and args.workload == "configs2" and not args.no_side:
        # the GPU is handed to the side runs: this job's buffers are released first
        oic.close()
        job.release()
        torch.cuda.empty_cache()
        side = side_runs()

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "overlaps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u8/2-bit bases, int32 edit rows", "data": "synthetic",
            "config": job.config(P_maxerate=job.P.maxErate, world=world, backend=backend),
            "overlaps_per_step": total_ovl,
            "parity": parity,
            "gbp_vs_gbp_per_sec": round(gbp_vs_gbp, 4),
            "breakdown_ms": {"index": round(st["ms_index"], 2), "seed": round(st["ms_seed"], 2),
                             "extend": round(st["ms_extend"], 2)},
            "seed_hits": st["seed_hits"], "seed_nodes": st["seed_nodes"], "pairs": st["pairs"],
            # overlapInCore's -s counters of the last step (rank 0's at N > 1) and the driver's
            # batch structure (hash batches, super-batches, query chunks)
            "counters": {k: st.get(k) for k in (
                "total_overlaps", "kmer_hits_with_olap", "kmer_hits_without_olap",
                "kmer_hits_skipped", "multi_overlaps", "contained_overlaps", "dovetail_overlaps",
                "hash_batches", "super_batches", "query_chunks", "sq_declined",
                "find_releases")},
            "pair_kernels": {"staged": st.get("staged_pairs"), "long": st.get("long_pairs"),
                             "generic": st.get("generic_pairs")},
            "setup_s": round(setup_s, 1),
            "setup_hbm": setup_hbm,
            "roofline": roof,
            "probe_roofline": probe_roof,
            "traffic_source": traffic_note,
            "seed_only": seed_only,
            "shard_timing": shard,
            "index_allgather": xgmi,
            "cpu_baseline": cpu,
        }
        if ovb is not None:
            line["ovb_output"] = ovb
        if side is not None:
            line.update(side)
        print(json.dumps(line), flush=True)
    oic.close()
    if dist:
        dist.destroy_process_group()


class Configs2:
    """BASELINE configs[2]: the all-vs-all job over one index, query shards per rank."""

    def __init__(self, args, rank, world, dev):
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        self.dist = None

    def release(self):
        """Drop the device copies of the read store (the context is closed by the caller)."""
        self._keep = None

    def workload_key(self) -> dict:
        a = self.args
        return {"workload": "configs2", "reads": a.reads, "read_len": a.read_len,
                "coverage": a.coverage, "read_error": a.read_error, "seed": a.seed, "k": a.k,
                "maxerate": float(np.float32(a.maxerate)), "minlength": a.minlength}

    def generate(self):
        """This rank's slice of the read set, on the host (no GPU call)."""
        from canu_amd.synth import synth_reads, random_genome
        a, n = self.args, self.args.reads
        genome_len = int(n * a.read_len / a.coverage)
        genome = random_genome(np.random.default_rng(a.seed), genome_len)
        lo = n * self.rank // self.world
        hi = n * (self.rank + 1) // self.world
        self._part = synth_reads(n_reads=n, read_len=a.read_len, genome_len=genome_len,
                                 error_rate=a.read_error, seed=a.seed, genome=genome,
                                 read_range=(lo, hi))

    def setup(self, OicParameters, OverlapInCore):
        import torch
        from canu_amd.dist import gather_read_store, query_shards
        a, n = self.args, self.args.reads
        part, self._part = self._part, None
        if self.world == 1:
            bases = torch.from_numpy(part.bases).to(self.dev)
            lengths = part.lengths
        else:
            bases, lengths = gather_read_store(torch.from_numpy(part.bases).to(self.dev),
                                               part.lengths, self.dist, self.dev)  # RCCL
        offsets = np.zeros(n, dtype=np.uint64)
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
        self._keep = (bases, torch.from_numpy(offsets.view(np.int64)).to(self.dev))
        self.total_bases = int(lengths.sum(dtype=np.uint64))
        self.nloaded = int(lengths.shape[0])
        self.n = n
        self.P = OicParameters(Kmer_Len=a.k, maxErate=float(np.float32(a.maxerate)),
                               Min_Olap_Len=a.minlength).finalize()
        self.oic = OverlapInCore(self.P, device=self.dev.index)
        self.oic.load_reads_device(1, bases.data_ptr(), self._keep[1].data_ptr(), lengths)
        torch.cuda.synchronize()
        self._keep = bases = None      # the library packed its own copy (load_common)
        torch.cuda.empty_cache()
        self.q_lo, self.q_hi = query_shards(n, self.world)[self.rank]

    # each rank indexes reads q_lo..n only: its queries' targets all have larger IDs
    # (Find_Overlaps.C:328), so records and counters equal the whole index's
    def step(self) -> int:
        self.oic.build_hash_index(self.q_lo, self.n)
        return self.oic.find_overlaps(self.q_lo, self.q_hi)

    def config(self, P_maxerate, world, backend):
        a = self.args
        return {"workload": "configs[2]: 50k synthetic ONT reads x 10 kb, full "
                            "overlapInCore (seed + banded extend), all-vs-all",
                "reads": a.reads, "read_len": a.read_len, "coverage": a.coverage,
                "read_error": a.read_error, "k": a.k, "maxerate": P_maxerate,
                "minlength": a.minlength, "parallelism": f"query-shard{world}",
                "dist_backend": backend if world > 1 else None}

    def parity(self, st, reduce, SUM, torch):
        """The last step's records (and -s counters) vs the reference's digest of the same
        reads, when this run's workload is the one the digest was made for."""
        from canu_amd import digest
        try:
            with open(GOLDEN) as f:
                g = json.load(f)
        except (OSError, ValueError):
            return {"checked": False, "reason": f"{os.path.relpath(GOLDEN, ROOT)} missing"}
        gw = g["workload"]
        mine = self.workload_key()
        same = all(np.isclose(float(gw[k]), float(mine[k])) for k in
                   ("reads", "read_len", "coverage", "read_error", "seed", "k", "maxerate",
                    "minlength"))
        t0 = time.time()
        rec = self.oic.fetch()
        mh = digest.multiset_hash(rec)
        if not same:       # still fingerprinted, so library variants can be compared
            return {"checked": False, "reason": "workload differs from the digest's",
                    "records": int(rec.shape[0]), "multiset_hash": f"{mh:016x}"}
        # the multiset hash adds up over the ranks' disjoint query shards; the sum is taken
        # as two 32-bit halves so the int64 all-reduce cannot overflow
        lo = int(reduce(mh & 0xFFFFFFFF, SUM, torch.int64))
        hi = int(reduce(mh >> 32, SUM, torch.int64))
        total_mh = (lo + (hi << 32)) & ((1 << 64) - 1)
        n_all = int(reduce(int(rec.shape[0]), SUM, torch.int64))
        names = {"kmer_hits_without_olap": "kmer_hits_without_olap",
                 "kmer_hits_with_olap": "kmer_hits_with_olap", "multi_overlaps": "multi",
                 "total_overlaps": "total", "contained_overlaps": "contained",
                 "dovetail_overlaps": "dovetail"}
        counters_ok = True
        for mine_k, ref_k in names.items():
            v = int(reduce(int(st[mine_k]), SUM, torch.int64))
            if v != int(g["stats"][ref_k]):
                counters_ok = False
        out = {"checked": True, "records": n_all, "ref_records": g["records"],
               "multiset_hash": f"{total_mh:016x}",
               "multiset_ok": f"{total_mh:016x}" == g["multiset_hash"],
               "counters_ok": counters_ok, "golden": os.path.relpath(GOLDEN, ROOT)}
        if self.world == 1:
            out["sha256_ok"] = digest.sha256_sorted(rec) == g["sha256_sorted"]
        out["ok"] = bool(out["multiset_ok"] and counters_ok and n_all == g["records"] and
                         out.get("sha256_ok", True))
        out["check_s"] = round(time.time() - t0, 2)
        return out

    def write_output(self, out_dir: str) -> dict:
        """This rank's output files as overlapInCore writes them with -o / -s
        (overlapInCore.C:197, :569): <dir>/<rank>.ovb (snappy-framed ovFile) + .counts, and
        the -s stats text -- timed from the device-resident records (fetch, host sort,
        encode, write).  The host merge of the ranks' files into one store is canu's own
        ovStoreBuild (tests/test_store_merge.py)."""
        os.makedirs(out_dir, exist_ok=True)
        base = os.path.join(out_dir, f"rank{self.rank:02d}")
        t0 = time.perf_counter()
        self.oic.write_ovb(base + ".ovb")
        t1 = time.perf_counter()
        self.oic.write_stats(base + ".stats")
        size = sum(os.path.getsize(base + x) for x in (".ovb", ".counts")
                   if os.path.exists(base + x))
        return {"ovb": os.path.relpath(base + ".ovb", ROOT) if base.startswith(ROOT) else
                base + ".ovb", "records": int(self.oic.stats()["total_overlaps"]),
                "bytes": size, "write_s": round(t1 - t0, 2),
                "note": "after the timed region: fetch + host sort + .ovb/.counts encode and "
                        "write of this rank's records (ovl_ctx_write_ovb)"}

    def seed_only(self):
        """BASELINE configs[1] on the same read set: the hash index + seed-hit kernels alone
        (the Add_Ref hit list of every query, both orientations, written to HBM)."""
        self.oic.build_hash_index(self.q_lo, self.n)
        n_hits = self.oic.seed_hits(self.q_lo, self.q_hi, fetch=False)
        st1 = self.oic.stats()
        return {"workload": "configs[1]: hash index + seed-hit list, same reads",
                "seed_hits": n_hits, "ms_index": round(st1["ms_index"], 2),
                "ms_seed_hits": round(st1["ms_seed_hits"], 2),
                "seed_hits_per_s": round(n_hits / ((st1["ms_index"] + st1["ms_seed_hits"])
                                                   * 1e-3), 1)}

    def shard_timing(self, ms_step):
        """The 8-way query shards (dist.query_shards) one after another on this GPU, each
        with its own index build, as each rank of an 8-GPU job runs them."""
        import torch
        from canu_amd.dist import query_shards
        shard_ms = []
        for lo8, hi8 in query_shards(self.n, 8):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            self.oic.build_hash_index(lo8, self.n)
            self.oic.find_overlaps(lo8, hi8)
            torch.cuda.synchronize()
            shard_ms.append(round(1000.0 * (time.perf_counter() - t1), 1))
        return {"shards": 8, "shard_ms": shard_ms,
                "projected_speedup_8": round(sum(shard_ms) / max(shard_ms), 2),
                "projected_vs_1gpu_step": round(ms_step / max(shard_ms), 2),
                "note": "the 8 ranks' jobs (index over the shard's lo..n, then its queries) "
                        "timed in turn on one GPU; projected_speedup_8 = sum / max, "
                        "projected_vs_1gpu_step = this run's 1-GPU step / the slowest rank; "
                        "the driver's 8-GPU run measures the real curve"}

    def index_allgather_timing(self, torch):
        """The north star's shared index, measured on this node: rank 0 builds the index over
        every read (1..n), and its buffers (ovl_export_index) go to the other ranks over RCCL
        (broadcast), which import them (ovl_import_index; dist.share_index) -- timed beside
        the index build each rank does instead over its shard's reads lo..n.  Then every rank
        searches its shard with the shared index: the records must equal its own step's."""
        from canu_amd import digest
        from canu_amd.dist import share_index
        st = self.oic.stats()
        own_mh = digest.multiset_hash(self.oic.fetch())
        from canu_amd.dist import _agree
        torch.cuda.synchronize()
        self.dist.barrier()
        t0 = time.perf_counter()
        ok = True
        if self.rank == 0:
            try:
                self.oic.build_hash_index(1, self.n)
            except Exception:                # noqa: BLE001 -- every rank raises below
                ok = False
        if not _agree(ok, self.dist, self.dev):
            raise RuntimeError("shared index: rank 0's build failed")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        nbytes = share_index(self.oic, [] if self.rank == 0 else [self.oic], self.dist,
                             self.dev)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        same = False
        try:
            self.oic.find_overlaps(self.q_lo, self.q_hi)
            same = digest.multiset_hash(self.oic.fetch()) == own_mh
        except Exception:                    # noqa: BLE001 -- reported as a mismatch
            same = False
        t = torch.tensor([1000.0 * (t1 - t0), 1000.0 * (t2 - t1), 0.0 if same else 1.0],
                         dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        build_ms, share_ms, bad = (float(x) for x in t.tolist())
        return {"index_bytes": nbytes, "rank0_full_build_ms": round(build_ms, 2),
                "broadcast_import_ms": round(share_ms, 2),
                "shared_index_ms": round(build_ms + share_ms, 2),
                "rank_index_build_ms": round(st["ms_index"], 2),
                "records_equal_own_index": bad == 0.0,
                "note": "shared: rank 0 builds the whole index, RCCL broadcast of its buffers, "
                        "import on every rank (max over ranks); own: each rank's build over its "
                        "shard's reads lo..n (this rank's last step)"}


class Configs4Rank(Configs2):
    """One rank's job of configs[4]'s plan (4M x 12 kb on 8 GPUs) at 1/8 scale: the hash
    block `-h lo-hi` searched by `-r 1-hi`, OverlapDriver batches inside (overlapInCore.C:
    191-300) with canu's --hashbits 23 --hashload 0.75.  At N ranks the plan has N jobs and
    rank r runs job r; on one GPU `--rank-job` picks one of the 8-way plan's jobs."""

    HASHBITS, HASHLOAD = 23, 0.75

    def workload_key(self) -> dict:
        a = self.args
        return {"workload": "configs4-rank", "reads": a.reads, "read_len": a.read_len,
                "coverage": a.coverage, "read_error": a.read_error, "seed": a.seed, "k": a.k,
                "maxerate": float(np.float32(a.maxerate)), "minlength": a.minlength,
                "rank_job": a.rank_job,
                **({"plan": "r06"} if self.plan() == "r06" else {})}

    def plan(self) -> str:
        """Which cost model cuts the rank plan: "r06" (dist.DRIVER6: the driver's own
        super-batch / query-chunk planning replayed per job, round 6) at the full 4M-read
        size, "r02" (the rehearsal costs, the plan the committed 20k / 500k reference digests
        pin) below it; CANU_C4_PLAN overrides."""
        e = os.environ.get("CANU_C4_PLAN")
        if e in ("r02", "r06"):
            return e
        return "r06" if self.args.reads >= 4_000_000 else "r02"

    def plan_jobs(self):
        """The plan's jobs and this rank's job (self.jobs, self.job), from the workload's
        parameters alone (no reads, no GPU)."""
        from canu_amd.dist import c4_plan, hash_block_jobs
        a, n = self.args, self.args.reads
        plan_ranks = 8 if self.world == 1 else self.world
        load = self.HASHLOAD * (1 << self.HASHBITS) * 21
        if self.plan() == "r06":
            self.jobs = c4_plan(n, plan_ranks, a.read_len)
        else:
            self.jobs = hash_block_jobs(n, plan_ranks, a.read_len, 36.0, 3.0 * load)
        self.job = self.jobs[a.rank_job if self.world == 1 else self.rank]
        if os.environ.get("CANU_C4_HBLOCK"):          # "lo-hi": one job outside the plan (A/B)
            lo_h, hi_h = (int(x) for x in os.environ["CANU_C4_HBLOCK"].split("-"))
            self.job = {"h": (lo_h, hi_h), "r": (1, hi_h), "est_s": None}
        return self.jobs, self.job

    def generate(self):
        """This rank's slice of the read set, on the host before any GPU call (the
        generator's worker pool is forked here)."""
        from canu_amd.synth import synth_reads_parallel
        a, n = self.args, self.args.reads
        genome_len = int(n * a.read_len / a.coverage)
        self.plan_jobs()
        lo = n * self.rank // self.world
        hi = n * (self.rank + 1) // self.world
        if self.world == 1:
            # one GPU runs one job of the plan: only the reads it touches (1..max(h, r)) are
            # generated and loaded; the genome is the whole read set's, so they are the same
            # reads as in the full set (read i depends on (seed, i) and the genome alone)
            hi = max(self.job["h"][1], self.job["r"][1])
        # CANU_C4_READS_CACHE=<dir> (one rank): the read set saved there once and loaded by
        # later runs (saves the generation's ~10 s in repeated PMC passes)
        cache = os.environ.get("CANU_C4_READS_CACHE") if self.world == 1 else None
        key = f"c4_{n}_{hi}_{a.read_len}_{a.coverage}_{a.read_error}_{a.seed}"
        if cache and os.path.exists(os.path.join(cache, key + "_lengths.npy")):
            from canu_amd.synth import ReadSet
            lens = np.load(os.path.join(cache, key + "_lengths.npy"))
            offs = np.zeros(lens.shape[0], dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
            part = ReadSet(bases=np.load(os.path.join(cache, key + "_bases.npy")),
                           offsets=offs, lengths=lens)
        else:
            part = synth_reads_parallel(n, a.read_len, genome_len, a.read_error, seed=a.seed,
                                        len_jitter=0.2, read_range=(lo, hi),
                                        workers=max(1, 16 // self.world))
            if cache:
                os.makedirs(cache, exist_ok=True)
                np.save(os.path.join(cache, key + "_bases.npy"), part.bases)
                np.save(os.path.join(cache, key + "_lengths.npy"), part.lengths)
        self._part = part

    def setup(self, OicParameters, OverlapInCore):
        import torch
        from canu_amd.dist import gather_read_prefix
        a, n = self.args, self.args.reads
        part, self._part = self._part, None
        if self.world == 1:
            bases = torch.from_numpy(part.bases).to(self.dev)
            lengths = part.lengths
        else:
            # each rank receives only reads 1..max(h, r) -- what its job touches, as the
            # one-GPU runs load -- point to point from the ranks that generated them
            need = max(self.job["h"][1], self.job["r"][1])
            local = torch.from_numpy(part.bases).to(self.dev)
            bases, lengths = gather_read_prefix(local, part.lengths, need, self.dist, self.dev)
            del local
        del part
        offsets = np.zeros(lengths.shape[0], dtype=np.uint64)
        offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
        self._keep = (bases, torch.from_numpy(offsets.view(np.int64)).to(self.dev))
        self.total_bases = int(lengths.sum(dtype=np.uint64))
        self.nloaded = int(lengths.shape[0])
        self.n = n
        (h_lo, h_hi), (r_lo, r_hi) = self.job["h"], self.job["r"]
        hashed = int(lengths[h_lo - 1:h_hi].sum(dtype=np.uint64)) + (h_hi - h_lo + 1)
        self.P = OicParameters(Kmer_Len=a.k, maxErate=float(np.float32(a.maxerate)),
                               Min_Olap_Len=a.minlength, bgnHashID=h_lo, endHashID=h_hi,
                               bgnRefID=r_lo, endRefID=r_hi, Hash_Mask_Bits=self.HASHBITS,
                               Max_Hash_Load=self.HASHLOAD, Max_Hash_Strings=10_000_000,
                               Max_Hash_Data_Len=hashed + 1024, Num_PThreads=16).finalize()
        self.oic = OverlapInCore(self.P, device=self.dev.index)
        self.oic.load_reads_device(1, bases.data_ptr(), self._keep[1].data_ptr(), lengths)
        torch.cuda.synchronize()
        # the library packed its own 2-bit copy (load_common) and never reads these bases
        # again: the 1-B-per-base staging (48 GB at 4M x 12 kb) goes back to the device
        # before the driver sizes its super-batches and query chunks from free HBM
        self._keep = bases = None
        torch.cuda.empty_cache()

    def step(self) -> int:
        return self.oic.overlap_driver(store_num_reads=self.n)

    def config(self, P_maxerate, world, backend):
        a = self.args
        scale = "full scale" if a.reads >= 4_000_000 else f"{a.reads / 4e6:g} scale"
        return {"workload": f"configs[4] rank job at {scale}: {a.reads // 1000}k ONT reads x "
                            f"{a.read_len // 1000} kb (+-20 %) at {a.coverage:g}x, one "
                            "`-h lo-hi -r 1-hi` OverlapDriver job of the "
                            f"{len(self.jobs)}-rank plan, --hashbits {self.HASHBITS} "
                            f"--hashload {self.HASHLOAD}",
                "reads": a.reads, "read_len": a.read_len, "coverage": a.coverage,
                "read_error": a.read_error, "k": a.k, "maxerate": P_maxerate,
                "minlength": a.minlength, "job": {"h": list(self.job["h"]),
                                                  "r": list(self.job["r"]),
                                                  "index": a.rank_job if world == 1 else "rank"},
                "hash_batches": self.oic.stats()["hash_batches"],
                "parallelism": f"hash-block{world}",
                "dist_backend": backend if world > 1 else None}

    def parity(self, st, reduce, SUM, torch):
        """Each rank's job vs the reference's digest of the same plan job
        (tests/golden/c4rank<reads/1000>k.json, tools/make_c4_digest.py), when one was made
        for this read set; the 1/8-scale default has none (the reference would take hours)."""
        from canu_amd import digest
        a = self.args
        path = os.path.join(ROOT, "tests", "golden", f"c4rank{a.reads // 1000}k.json")
        g = None
        try:
            with open(path) as f:
                g = json.load(f)
        except (OSError, ValueError):
            pass
        mine = self.workload_key()
        same = g is not None and all(
            np.isclose(float(g["workload"][k]), float(mine[k])) for k in
            ("reads", "read_len", "coverage", "read_error", "seed", "k", "maxerate",
             "minlength"))
        gj = None
        if same:
            for j in g["jobs"]:
                if tuple(j["h"]) == tuple(self.job["h"]) and tuple(j["r"]) == tuple(self.job["r"]):
                    gj = j
        # every rank must agree on whether the check runs (the reduces below are collective)
        have = int(reduce(1 if gj is not None else 0, SUM, torch.int64))
        if have != self.world:
            return {"checked": False, "reason": "no reference digest for this plan job "
                    "(tools/make_c4_digest.py pins the 20k-read plan; the rank-job union and "
                    "oic_ref parity are tests/test_configs4.py, -m gpu)"}
        t0 = time.time()
        rec = self.oic.fetch()
        names = {"kmer_hits_without_olap": "kmer_hits_without_olap",
                 "kmer_hits_with_olap": "kmer_hits_with_olap", "multi_overlaps": "multi",
                 "total_overlaps": "total", "contained_overlaps": "contained",
                 "dovetail_overlaps": "dovetail"}
        ok = (rec.shape[0] == gj["records"] and
              digest.sha256_sorted(rec) == gj["sha256_sorted"] and
              f"{digest.multiset_hash(rec):016x}" == gj["multiset_hash"] and
              all(int(st[m]) == int(gj["stats"][r]) for m, r in names.items()))
        n_ok = int(reduce(1 if ok else 0, SUM, torch.int64))
        return {"checked": True, "ok": n_ok == self.world, "jobs_ok": n_ok,
                "records": int(reduce(int(rec.shape[0]), SUM, torch.int64)),
                "golden": os.path.relpath(path, ROOT), "check_s": round(time.time() - t0, 2)}

    def seed_only(self):
        return None

    def shard_timing(self, ms_step):
        return None

    def index_allgather_timing(self, torch):
        return None


def source_hash() -> str:
    """SHA-256 (16 hex) of the HIP sources the PMC counters were taken from."""
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "canu_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.startswith("ovl_") and (name.endswith(".hip") or name.endswith(".h")):
            with open(os.path.join(csrc, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def load_traffic(job, world: int):
    """Per-kernel PMC figures (profiles/traffic*.json, tools/pmc_traffic.py) when they were
    taken on THIS workload (one rank) and THESE sources; else ({}, why not)."""
    fname = TRAFFIC_FILES[job.args.workload]
    path = os.path.join(ROOT, "profiles", fname)
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return {}, f"profiles/{fname} missing"
    meta = t.get("_method", {})
    if world != 1:
        return {}, "PMC counters are per-workload single-GPU figures: not used at N > 1"
    if meta.get("workload") != job.workload_key():
        return {}, f"PMC passes ({meta.get('tag')}) were taken on another workload"
    if meta.get("src_sha") != source_hash():
        return {}, f"PMC passes ({meta.get('tag')}) were taken on other kernel sources"
    return t, f"profiles/{fname} ({meta.get('tag')}, same workload and sources)"


def rooflines(args, job, st, world):
    """The dominant kernel (k_extend) against the roofline that binds it -- instruction
    issue -- with its HBM figures beside; and the hash-probe kernel against HBM."""
    traffic, note = load_traffic(job, world)
    n = job.n
    avg_len = job.total_bases / max(job.nloaded, 1)
    strand = 8.0 * (np.ceil(avg_len / 32.0) + 1.0)
    # algorithmic HBM bytes of k_extend per pair: both packed strands, 16 B per seed-match
    # node (the Add_Match lists), 24 B per record written
    ext_bytes = st["pairs"] * 2 * strand + st["seed_nodes"] * 16 + st["total_overlaps"] * 24
    roof = None
    n_ext = max(int(st.get("extend_launches", 0)), 1)
    if st["ms_extend"] > 0:
        per_launch = ext_bytes / n_ext
        avg_ms = st["ms_extend"] / n_ext
        hbm_gbs = per_launch / (avg_ms * 1e-3) / 1e9
        ext = traffic.get("k_extend", {})
        tb = ext.get("hbm_bytes_per_launch")
        hbm = {"achieved": round(hbm_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hbm_gbs / HBM_PEAK_GBS, 5), "traffic": tb,
               "traffic_gbs": round(tb / (avg_ms * 1e-3) / 1e9, 1) if tb else None,
               "traffic_frac": round(tb / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
               if tb else None}
        iss = ext.get("issue")
        roof = {"kernel": "k_extend", "algorithmic_bytes_per_launch": int(per_launch),
                "launches": n_ext, "avg_launch_ms": round(avg_ms, 3)}
        if iss:
            # wave-instructions per launch from PMC (deterministic for a workload and build)
            # over this run's launch time, against the issue peaks: one SALU per CU-cycle
            # (one scalar unit per CU), one VALU per 2 cycles per SIMD (wave64 on SIMD-32)
            launches = ext.get("launches_per_step", 1)
            secs = avg_ms * 1e-3
            salu = iss["salu_insts"] / launches / secs / 1e9
            valu = iss["valu_insts"] / launches / secs / 1e9
            salu_pk = N_CU * CLOCK_GHZ
            valu_pk = N_SIMD * CLOCK_GHZ / 2.0
            bind = "SALU" if salu / salu_pk >= valu / valu_pk else "VALU"
            a, p = (salu, salu_pk) if bind == "SALU" else (valu, valu_pk)
            roof.update({"bound": "issue", "achieved": round(a, 1), "peak": round(p, 1),
                         "unit": f"G {bind} wave-instructions/s", "frac": round(a / p, 4),
                         "traffic": tb, "binding_unit": bind,
                         "salu_frac": round(salu / salu_pk, 4),
                         "valu_frac": round(valu / valu_pk, 4), "hbm": hbm,
                         "limiter": "instruction issue of the greedy O(ND) rows: integer "
                                    "VALU and the per-row scalar control at about equal "
                                    "shares of their peaks; 6 waves per SIMD (LDS-capped), "
                                    "and 8 measured no faster (DESIGN.md round 4), so the "
                                    "waves' dependency chains are covered and the row's "
                                    "instruction count is what binds.  HBM moves the row log "
                                    "and spills (hbm.traffic_gbs), not the algorithmic bytes"})
        else:
            roof.update({"bound": "hbm", "achieved": hbm["achieved"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": hbm["frac"], "traffic": None,
                         "limiter": "issue-bound (see DESIGN.md); no PMC issue counters "
                                    "for this workload/build, so the HBM figure is given"})
    probe_roof = None
    n_pr = max(int(st.get("probe_launches", 0)), 1)
    if st["ms_probe_kernel"] > 0:
        per_launch = st["probe_bytes"] / n_pr
        avg_ms = st["ms_probe_kernel"] / n_pr
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        n_sorted = int(st.get("probe_sorted_launches", 0))
        kname = "k_probe_sorted" if n_sorted == n_pr else "k_probe" if n_sorted == 0 else \
            "k_probe + k_probe_sorted"
        tb = traffic.get(kname, {}).get("hbm_bytes_per_launch")
        probe_roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                      "traffic": tb, "kernel": kname,
                      "algorithmic_bytes_per_launch": int(per_launch), "launches": n_pr,
                      "avg_launch_ms": round(avg_ms, 3)}
        if n_sorted:
            # the sorted-window probe streams the job's sorted windows, the table and its
            # filter (12 B per window + the table's and filter's bytes, hit records not
            # counted): an HBM stream, not random lookups, so the random-lookup ceilings
            # below do not bound it
            probe_roof["sorted_launches"] = n_sorted
            probe_roof["note"] = ("k_probe_sorted (the job's windows sorted by k-mer, DESIGN.md "
                                  "round 4): bytes = 12 per sorted window + the table and "
                                  "filter read once, or at most one 16-B entry and one 8-B "
                                  "filter word per window when they are larger than the run "
                                  "(round 5); it does no random table lookups, so it is "
                                  "priced against HBM only")
            return roof, probe_roof, note
        if tb:
            probe_roof["traffic_gbs"] = round(tb / (avg_ms * 1e-3) / 1e9, 1)
            probe_roof["traffic_frac"] = round(probe_roof["traffic_gbs"] / HBM_PEAK_GBS, 4)
        wps = achieved * 1e9 / PROBE_BYTES_PER_WINDOW
        # the ceiling of one random lookup per window, measured now on this device over this
        # run's own index table (ovl_probe_ceiling: 8 independent random 16-B loads in flight
        # per lane, nothing else in the loop)
        ceil = {"windows_per_s": round(wps / 1e9, 2)}
        try:
            g, tbytes = job.oic.probe_ceiling()
            ceil.update({"ceiling_gloads_per_s": round(g, 2), "table_bytes": int(tbytes),
                         "frac_of_ceiling": round(wps / 1e9 / g, 3) if g > 0 else None,
                         "source": "live: ovl_probe_ceiling over this run's index table"})
            if g > 0 and wps / 1e9 > g:
                ceil["note"] = ("the probe beats uniform random loads here: its lookups are not "
                                "uniform over the table (repeated k-mers hit cached lines); "
                                "the replay below is the ceiling for its own lookups")
            # the probe's own lookup stream (the job's query windows, first 2^28) replayed as
            # pure loads over the same table (ovl_probe_replay): the rate the memory system
            # gives these exact lookups, so frac_of_replay is the probe's overhead over them
            if getattr(job, "q_lo", None) is not None:
                gr, nw = job.oic.probe_replay(job.q_lo, job.q_hi)
                ceil.update({"replay_gloads_per_s": round(gr, 2), "replay_windows": int(nw),
                             "frac_of_replay": round(wps / 1e9 / gr, 3) if gr > 0 else None,
                             "replay_source": "live: ovl_probe_replay, the probe's own slots"})
        except Exception as e:        # a side figure: never lose the bench line to it
            ceil["error"] = f"{type(e).__name__}: {e}"[:200]
        probe_roof["random_lookup_ceiling"] = ceil
    return roof, probe_roof, note


def side_runs(timeout_s: int = 300) -> dict:
    """The other two workloads BASELINE.json names, each timed by its own bench in a child
    process on this GPU after the headline (one warm-up + one timed job each), so the
    driver's default run records them too; the headline's value is not touched:
      configs4_rank  bench.py --workload configs4-rank (one rank job of configs[4]'s 8-GPU
                     plan at 1/8 scale, with its PMC-keyed issue roofline when
                     profiles/traffic_configs4.json matches these sources)
      mhap_configs3  bench_mhap.py (configs[3]: 200k x 15 kb, canu's weighting; parity with
                     the MHAP jar unpinned)"""
    import subprocess
    keep4 = ("value", "unit", "ms_per_step", "breakdown_ms", "pairs", "pair_kernels",
             "roofline", "probe_roofline", "traffic_source", "config", "setup_s", "setup_hbm",
             "parity", "counters", "ovb_output")
    keep3 = ("value", "unit", "ms_per_step", "breakdown_ms", "config", "setup_s", "roofline",
             "candidates_per_step", "overlaps_per_step", "parity")
    runs = {"configs4_rank": ([sys.executable, os.path.join(ROOT, "bench.py"), "--workload",
                               "configs4-rank", "--steps", "1", "--warmup", "1",
                               "--no-cpu-baseline", "--no-side"], keep4),
            "mhap_configs3": ([sys.executable, os.path.join(ROOT, "bench_mhap.py"), "--steps",
                               "1", "--warmup", "1", "--no-cpu-baseline"], keep3)}
    out = {}
    for name, (cmd, keep) in runs.items():
        t0 = time.time()
        try:
            cp = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
            lines = [l for l in cp.stdout.splitlines() if l.startswith("{")]
            if cp.returncode != 0 or not lines:
                out[name] = {"error": f"rc {cp.returncode}: {cp.stderr[-300:]}"}
                continue
            d = json.loads(lines[-1])
            out[name] = {k: d[k] for k in keep if k in d}
            out[name]["wall_s"] = round(time.time() - t0, 1)
        except Exception as e:                  # never lose the headline to a side run
            out[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
    return out


def cpu_share() -> dict:
    """The CPUs this process may use: the cgroup quota (cpu.max) and the affinity mask."""
    out = {"host_cpus": os.cpu_count()}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        out["affinity"] = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        out["cgroup_cpu_max"] = f"{q} {per}"
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        out["cgroup_cpu_max"] = None
    out["quota_cpus"] = quota
    usable = out["affinity"] or 1
    if quota is not None:
        usable = min(usable, max(1, int(quota)))
    out["usable"] = usable
    return out


def cpu_baseline(args) -> dict | None:
    """The reference overlapInCore (oracle/_ref/oic_ref, built from its sources) on a
    bounded sample of the same workload: fewer reads, same read length / error / coverage,
    canu's production hash settings -- utgOvlHashBits 23, utgOvlHashLoad 0.75
    (Defaults.pm:687-688) -- and the sample split into --cpu-batches hash batches
    (--hashstrings), as canu's jobs are.  Threads: min(64, the CPUs this process may use:
    cgroup quota and affinity); a 64-core figure is only reported when 64 were usable."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import oracle
        from canu_amd.synth import synth_reads
    except Exception:
        return None
    if not oracle.reference_available():
        return None
    share = cpu_share()
    threads = max(1, min(args.cpu_max_threads, share["usable"]))
    ns = args.cpu_sample_reads
    gl = int(ns * args.read_len / args.coverage)
    rs = synth_reads(ns, args.read_len, gl, args.read_error, seed=args.seed + 1000)
    p = oracle.default_params(kmer_len=args.k, max_erate=args.maxerate,
                              min_olap_len=args.minlength)
    # hash batches by --hashstrings (a --hashdatalen below the range's bases trips the
    # reference's assert at Build_Hash_Index.C:523)
    nb = max(1, args.cpu_batches)
    strings = (rs.nreads + nb - 1) // nb
    datalen = rs.total_bases() + rs.nreads + 1
    rec, secs, wall = oracle.run_reference(
        rs, p, threads=threads, hash_bits=23, with_time=True,
        batching={"hashstrings": strings, "hashdatalen": datalen, "hashload": 0.75})
    v = len(rec) / secs
    out = {"value": round(v, 1), "unit": "overlaps/s", "cores": threads,
           "kind": "reference", "per_core": round(v / threads, 1), "cpu_share": share,
           "sample": f"{ns} reads x {args.read_len} bp at {args.coverage:.0f}x "
                     f"(genome {gl} bp), --hashbits 23 --hashload 0.75 --hashstrings "
                     f"{strings} ({nb} hash batches), -t {threads}, reference OverlapDriver() "
                     f"wall {secs:.2f}s incl. its .ovb writing, {len(rec)} overlaps"}
    if threads >= 64:
        out["host64_measured"] = round(v, 1)
    else:
        out["host64_measured"] = None
        out["host64_note"] = (f"{threads}-core share of this host (cgroup/affinity); a 64-core "
                              "figure was not measurable here")
    return out


if __name__ == "__main__":
    main()
