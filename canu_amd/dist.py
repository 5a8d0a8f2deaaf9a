"""Multi-GPU layout of one overlapInCore job: one process per GPU.

The reference splits an all-vs-all job into independent overlapInCore runs, each over a
hash range (-h) and a query range (-r), scheduled by overlapInCorePartition
(src/overlapInCore/overlapInCorePartition.C).  Here every rank holds the whole read store
in HBM (288 GB holds any realistic batch), builds the same index over -h, and searches its
own query shard of -r: shards are independent, so the data path has no collective.  The
only exchange is at setup, when the ranks that each generated (or read) a slice of the
store all-gather it -- over RCCL/xGMI on the GPUs, over gloo in the CPU tests.
"""
from __future__ import annotations

import numpy as np


# The cost model of one rank's job, from the 1-GPU step on 50k x 10 kb (1 MI355X; round 5,
# profiles/r05c_bench.json: index 29 ms over every hashed read, probe 29 ms and chain
# 62 ms over every query, extension 1,037 ms over the n^2/2 (a, b > a) pairs).  A query shard [lo, hi] only ever pairs with reads
# b > a >= lo (Find_Overlaps.C:328 keeps targets with a larger ID), so its rank indexes
# reads lo..n only: the same records and counters, a smaller index, and occurrence lists
# (chain work) shortened by (n - lo) / n.
# One exception: under -l (Frag_Olap_Limit) the order a query's targets are processed in
# comes from String_Olap_Space slots that hash the target's number WITHIN the hash batch
# (Find_Overlaps.C:158-200), so a shard indexing lo..n reproduces the reference's
# `-h lo-n -r lo-hi` job exactly, not `-h 1-n`: once a limit is reached, other overlaps may
# be kept.  canu never passes -l to overlapInCore; bench.py does not use it.
SHARD_COSTS = {"index_per_read": 29.0 / 50_000, "probe_per_query": 29.0 / 50_000,
               "chain_per_query": 62.0 / 50_000, "pair": 1037.0 / (50_000 ** 2 / 2)}


def shard_cost(n: int, lo: int, hi: int, costs: dict | None = None) -> float:
    """Modelled time of the rank searching queries lo..hi (index over lo..n)."""
    c = SHARD_COSTS if costs is None else costs
    if hi < lo:
        return 0.0
    q = hi - lo + 1
    hashed = n - lo + 1
    pairs = q * (2 * n - lo - hi) / 2.0                # sum of n - a over the shard
    return (c["index_per_read"] * hashed + c["probe_per_query"] * q +
            c["chain_per_query"] * q * hashed / n + c["pair"] * pairs)


def query_shards(n: int, world: int, first: int = 1,
                 costs: dict | None = None) -> list[tuple[int, int]]:
    """Split query IDs first..first+n-1 into `world` contiguous shards of equal modelled
    time (shard_cost: each rank indexes its own lo..n).  Ranges are inclusive and may be
    empty (lo > hi) when world > n."""
    if n <= 0:
        return [(first, first - 1)] * world

    def cut(target: float) -> list[int]:
        ends, lo = [], 1
        for _ in range(world - 1):
            a, b = lo - 1, n
            while a < b:                               # largest hi with cost <= target
                mid = (a + b + 1) // 2
                if shard_cost(n, lo, mid, costs) <= target:
                    a = mid
                else:
                    b = mid - 1
            ends.append(a)
            lo = a + 1
        ends.append(n)
        return ends

    lo_t, hi_t = 0.0, shard_cost(n, 1, n, costs)
    for _ in range(60):
        mid = (lo_t + hi_t) / 2.0
        ends = cut(mid)
        last_lo = ends[-2] + 1 if world > 1 else 1
        if shard_cost(n, last_lo, n, costs) <= mid:
            hi_t = mid
        else:
            lo_t = mid
    out, lo = [], 1
    for hi in cut(hi_t):
        out.append((first - 1 + lo, first - 1 + hi))
        lo = hi + 1
    return out


def _all_gather(dist, out_list, t):
    """all_gather that also works on a CPU-only backend (gloo) with device tensors: those
    are staged through host memory (rehearsals only; RCCL gathers in HBM)."""
    if t.is_cuda and dist.get_backend() == "gloo":
        host = [o.cpu() for o in out_list]
        dist.all_gather(host, t.cpu())
        for o, h in zip(out_list, host):
            o.copy_(h)
    else:
        dist.all_gather(out_list, t)


def gather_read_store(bases_local, lengths_local: np.ndarray, dist, device):
    """All-gather every rank's slice of the read store (rank order = read order).

    bases_local: 1-D uint8 torch tensor on `device`; lengths_local: uint32 numpy array.
    Returns (bases, lengths): the whole store as a uint8 tensor on `device` and a uint32
    numpy array of read lengths."""
    import torch
    world = dist.get_world_size()
    n_b = torch.tensor([bases_local.numel()], device=device, dtype=torch.int64)
    n_l = torch.tensor([lengths_local.shape[0]], device=device, dtype=torch.int64)
    all_nb = [torch.zeros_like(n_b) for _ in range(world)]
    all_nl = [torch.zeros_like(n_l) for _ in range(world)]
    _all_gather(dist, all_nb, n_b)
    _all_gather(dist, all_nl, n_l)
    nbs = [int(x.item()) for x in all_nb]
    nls = [int(x.item()) for x in all_nl]
    buf = torch.zeros(max(nbs), dtype=torch.uint8, device=device)
    buf[:bases_local.numel()] = bases_local
    got = [torch.empty(max(nbs), dtype=torch.uint8, device=device) for _ in range(world)]
    _all_gather(dist, got, buf)
    bases = torch.cat([g[:k] for g, k in zip(got, nbs)])
    lb = torch.zeros(max(nls), dtype=torch.int64, device=device)
    lb[:lengths_local.shape[0]] = torch.from_numpy(lengths_local.astype(np.int64)).to(device)
    gl = [torch.empty(max(nls), dtype=torch.int64, device=device) for _ in range(world)]
    _all_gather(dist, gl, lb)
    lengths = torch.cat([g[:k] for g, k in zip(gl, nls)]).cpu().numpy().astype(np.uint32)
    return bases, lengths


def gather_read_prefix(bases_local, lengths_local: np.ndarray, need: int, dist, device):
    """configs[4]'s setup exchange: every rank generated (or read) one slice of the store
    (rank order = read order), and rank r needs only reads 1..need_r -- the reads its
    `-h lo-hi -r 1-hi` job touches (a job never reads past its hash block's end).  Each slice
    goes point to point to the ranks that need part of it, straight into their buffers
    (RCCL send / recv over xGMI; gloo stages device tensors through host memory): no rank
    holds reads it does not search, and nothing but the result stays allocated.

    bases_local: 1-D uint8 torch tensor; lengths_local: uint32 numpy array; need: this rank's
    read count from read 1 (clipped to the store).  Returns (bases, lengths) of reads
    1..need: a uint8 tensor on `device` and a uint32 numpy array."""
    import torch
    world, rank = dist.get_world_size(), dist.get_rank()
    cpu_stage = dist.get_backend() == "gloo" and bases_local.is_cuda
    meta_dev = torch.device("cpu") if dist.get_backend() == "gloo" else device
    m = torch.tensor([lengths_local.shape[0], need], dtype=torch.int64, device=meta_dev)
    allm = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(allm, m)
    nls = [int(x[0]) for x in allm]
    needs = [int(x[1]) for x in allm]
    total = sum(nls)
    # every rank gets every read's length (4 B per read): the byte ranges follow from them
    lb = torch.zeros(max(nls), dtype=torch.int64, device=meta_dev)
    lb[:nls[rank]] = torch.from_numpy(lengths_local.astype(np.int64))
    gl = [torch.empty_like(lb) for _ in range(world)]
    dist.all_gather(gl, lb)
    lengths = torch.cat([g[:k] for g, k in zip(gl, nls)]).cpu().numpy().astype(np.uint32)
    del gl, lb
    cum = np.zeros(total + 1, dtype=np.uint64)
    cum[1:] = np.cumsum(lengths, dtype=np.uint64)
    first = np.zeros(world + 1, dtype=np.int64)
    first[1:] = np.cumsum(nls)
    needs = [min(max(x, 0), total) for x in needs]

    def part(s, r):            # bytes of slice s that rank r needs: [0, b) of s's bases
        end = min(int(first[s + 1]), needs[r])
        return int(cum[end] - cum[first[s]]) if end > first[s] else 0

    mine = needs[rank]
    out = torch.empty(int(cum[mine]), dtype=torch.uint8, device=device)
    ops, staged = [], []
    b = part(rank, rank)
    if b:
        out[int(cum[first[rank]]):int(cum[first[rank]]) + b].copy_(bases_local[:b])
    for r in range(world):
        b = part(rank, r)
        if r != rank and b:
            t = bases_local[:b]
            if cpu_stage:
                t = t.cpu()
            ops.append(dist.P2POp(dist.isend, t, r))
    for s in range(world):
        b = part(s, rank)
        if s != rank and b:
            o = int(cum[first[s]])
            dst = out[o:o + b]
            if cpu_stage:
                h = torch.empty(b, dtype=torch.uint8)
                staged.append((dst, h))
                dst = h
            ops.append(dist.P2POp(dist.irecv, dst, s))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for dst, h in staged:
        dst.copy_(h)
    if out.is_cuda:
        torch.cuda.synchronize(device)
    return out, lengths[:mine]


def read_slices(n: int, world: int) -> list[tuple[int, int]]:
    """[lo, hi) of the reads rank r generates / sketches: n * r // world .. n * (r+1) // world."""
    return [(n * r // world, n * (r + 1) // world) for r in range(world)]


def all_gather_rows(local, n: int, dist):
    """All-gather a per-rank slice of rows (torch tensor [rows_r, ...], slices as
    read_slices(n, world)) into the whole [n, ...] tensor, in rank order.  One collective:
    slices are padded to the largest one (RCCL over xGMI on the GPUs, gloo on CPU)."""
    import torch
    world = dist.get_world_size()
    sl = read_slices(n, world)
    rmax = max(hi - lo for lo, hi in sl)
    pad = torch.zeros((rmax,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    got = [torch.empty_like(pad) for _ in range(world)]
    _all_gather(dist, got, pad)
    return torch.cat([g[:hi - lo] for g, (lo, hi) in zip(got, sl)])


# configs[4] (4M x 12 kb on 8 GPUs): per-unit costs measured by tools/rehearse_configs4.py on
# one MI355X (500k x 12 kb, 15x, --hashbits 26 --hashload 0.75: 4 hash batches, 23.7 s):
#   extension  19.7 s for 9.0 M pairs       -> ~2.2 us per (a < b) candidate pair
#   seed        2.2 s for 48 G query windows probed (500k queries x 2 strands x ~12 k x 4)
#   index       1.4 s for 6 G hashed windows
REHEARSAL_COSTS = {"pair_s": 19.7 / 9.0e6, "probe_window_s": 2.2 / 48e9,
                   "index_window_s": 1.4 / 6.0e9}

# Round 6: the driver's own planning rules replayed per job (ovl_overlap_driver, ovl_api.hip),
# so that a plan sees the discrete steps -- hash batches packed whole into super-batches, the
# query range cut into chunks -- that round 5's continuous fit smoothed over (its last three
# boundaries were moved by hand below a packing step).  HBM figures are the device's and the library's own:
#   device 309.2 GB (hipMemGetInfo's total), read store 1.0 GB + 0.75 B per base
#     (r06a: 272.2 GB free after loading 4M reads, 295.3 GB after 1.449M)
#   hash batch: the table load, 0.75 x 2^23 x 21 = 132.1 M windows (distinct k-mers ~ windows
#     at 15x over 12 kb reads: 20 batches for 220 k reads, 131 for 1.449 M)
#   super-batch cap = 0.55 x (free - 64 GB) / 112 windows (index_window_cap, phase 2), batches
#     packed whole: r06a 1.033 G at 4M reads loaded (7 per super-batch), 1.146 G at 1.449M (8)
#   an index holds 86 B per window of its largest super-batch (r06a: 80 GB for 0.93 G)
#   query chunk cap = ((free at planning) / 2 - one run's sort scratch) x 0.9 / 13 windows
#     (plan_query_chunks: 5.75 G windows at rank 7 of 4M, 6.33 G at 1.449 M)
# and per-unit device costs from the per-search OVL_TIMING lines of the same two jobs
# (profiles/r06a{0,7}_c4full_timing.log): a chunk's keys + sort 3.0e-11 s per window, a search
# 2.3e-11 s per window of the runs it touches + 10 ms, a super-batch build 4.5e-11 s per
# hashed window, phase 1 8 ms per hash batch, extension 0.68 us per pair (78.9 candidate pairs
# per hashed read b, times b / n, at 15x).
DRIVER6 = {"model": "driver6", "hbm": 309.2e9, "store_fixed": 1.0e9, "store_per_base": 0.75,
           "batch_windows": 0.75 * (1 << 23) * 21, "sb_frac": 0.55, "sb_reserve": 64.0 * (1 << 30),
           "sb_b_per_window": 112.0, "index_b_per_window": 86.0,
           "sort_scratch": 24.0 * (1 << 29) + 8.0 * (1 << 20), "chunk_b_per_window": 13.0,
           "run_windows": float(1 << 29),
           "pair_s": 0.68e-6, "pairs_per_read": 78.9, "sort_s": 3.0e-11, "probe_s": 2.3e-11,
           "search_s": 0.010, "build_s": 4.5e-11, "batch_s": 0.008, "job_s": 1.0}


def driver_plan(n: int, read_len: float, lo: int, hi: int, c: dict | None = None,
                k: int = 22) -> dict:
    """The batch structure ovl_overlap_driver gives a `-h lo-hi -r 1-hi` job over reads of
    about read_len (1..hi loaded), and its modelled seconds (DRIVER6)."""
    c = DRIVER6 if c is None else c
    w = max(read_len - k + 1, 1.0)                   # windows per read and strand
    m = hi - lo + 1
    free = c["hbm"] - c["store_fixed"] - c["store_per_base"] * read_len * hi
    bw = c["batch_windows"]
    # the table load cuts full batches of bw windows; the last one holds what is left
    full, tail = divmod(m * w, bw)
    sizes = [bw] * int(full) + ([tail] if tail > 0 else [])
    n_batch = max(1, len(sizes))
    sb_cap = c["sb_frac"] * max(free - c["sb_reserve"], 0.0) / c["sb_b_per_window"]
    # phase 2's greedy packing of whole batches (a batch past the cap is a super-batch alone)
    sbs, cur = [], 0.0
    for b in sizes:
        if sbs and cur + b <= sb_cap:
            sbs[-1] += b
            cur += b
        else:
            sbs.append(b)
            cur = b
    n_sb = max(1, len(sbs))
    sb_max = max(sbs) if sbs else 0.0
    sb_ends = np.cumsum(sbs) / w if sbs else np.array([float(m)])   # hashed reads, cumulative
    free_plan = free - c["index_b_per_window"] * sb_max
    budget = max((free_plan / 2.0 - c["sort_scratch"]) * 0.9, 0.0)
    ch_cap = max(budget / c["chunk_b_per_window"], 2.0 * w)
    ch_reads = max(1, int(ch_cap // (2.0 * w)))
    n_ch = -(-hi // ch_reads)
    searches, searched, built = 0, 0.0, 0.0
    for q in range(n_ch):
        q0, q1 = 1 + q * ch_reads, min(hi, (q + 1) * ch_reads)
        for s in range(n_sb):
            s0 = lo + (int(sb_ends[s - 1]) if s else 0)
            s1 = min(hi, lo + int(sb_ends[s]) - 1) if s + 1 < n_sb else hi
            if q0 < s1:
                searches += 1
                # the runs holding the chunk's reads below the super-batch's last read
                win = 2.0 * w * (min(q1, s1 - 1) - q0 + 1)
                searched += min(2.0 * w * (q1 - q0 + 1), win + c["run_windows"] / 2.0)
                built += w * (s1 - s0 + 1)
    pairs = c["pairs_per_read"] * m * (lo + hi) / 2.0 / n
    secs = (pairs * c["pair_s"] + 2.0 * w * hi * c["sort_s"] + searched * c["probe_s"] +
            searches * c["search_s"] + built * c["build_s"] + n_batch * c["batch_s"] + c["job_s"])
    return {"hash_batches": n_batch, "super_batches": n_sb, "query_chunks": n_ch,
            "searches": searches, "sb_cap": sb_cap, "chunk_cap": ch_cap, "pairs": pairs,
            "est_s": secs}


def c4_plan(n: int, world: int, read_len: float) -> list[dict]:
    """configs[4]'s plan at its real size: the blocks cut on DRIVER6 (the driver's packing
    replayed per job), in hash_block_jobs' format."""
    return hash_block_jobs(n, world, read_len, 36.0, 1.0, costs=DRIVER6)


def hash_block_jobs(n: int, world: int, read_len: float, pairs_per_read: float,
                    batch_windows: float, costs: dict | None = None) -> list[dict]:
    """canu's partitioning model with GPU-sized blocks: rank r runs ONE overlapInCore job
    (`-h lo_r-hi_r -r 1-hi_r`, the reference's OverlapDriver batches inside it) over a
    contiguous hash block; every (a < b) pair is found by the rank whose block holds b.
    pairs_per_read: candidate partners of a read among all reads (both sides; 36 for the
    rehearsal's 15x), of which read b has ~b / n before it.  Block r's work: its hashed
    reads' pairs with earlier reads, its index batches (batch_windows k-mers each), and
    every query a <= hi_r probing each batch.  Blocks
    are cut so the ranks' modelled times agree (the triangular pair count makes the first
    block the widest).  Returns per rank {"h": (lo, hi), "r": (1, hi), "est_s": seconds}."""
    c = dict(REHEARSAL_COSTS if costs is None else costs)
    w = max(read_len - 21.0, 1.0)                 # windows per read and strand (k = 22)

    def cost(lo: int, hi: int) -> float:
        if hi < lo:
            return 0.0
        if c.get("model") == "driver6":
            return driver_plan(n, read_len, lo, hi, c)["est_s"]
        m = hi - lo + 1
        pairs = pairs_per_read * (lo + hi) / 2.0 * m / n    # sum over b of b * ppr / n
        batches = max(1.0, m * w / batch_windows)
        probe = hi * 2.0 * w * batches
        return (pairs * c["pair_s"] + probe * c["probe_window_s"] +
                m * w * c["index_window_s"])

    def cut(target: float) -> list[int]:
        ends, lo = [], 1
        for _ in range(world - 1):
            a, b = lo - 1, n
            while a < b:                            # largest hi with cost(lo, hi) <= target
                mid = (a + b + 1) // 2
                if cost(lo, mid) <= target:
                    a = mid
                else:
                    b = mid - 1
            ends.append(a)
            lo = a + 1
        ends.append(n)
        return ends

    lo_t, hi_t = 0.0, cost(1, n)
    for _ in range(60):                             # the smallest target the last rank meets
        mid = (lo_t + hi_t) / 2.0
        ends = cut(mid)
        lo_last = (ends[-2] + 1) if world > 1 else 1
        if cost(lo_last, n) <= mid:
            hi_t = mid
        else:
            lo_t = mid
    ends = cut(hi_t)
    jobs, lo = [], 1
    for hi in ends:
        jobs.append({"h": (lo, hi), "r": (1, hi), "est_s": round(cost(lo, hi), 2)})
        lo = hi + 1
    return jobs


# ---- one index shared by the ranks (the north star's "all-gather the index over xGMI") ----
_INDEX_PARTS = ("table", "occ", "bloom", "read_flags")
_INDEX_META = ("bgn_iid", "end_iid", "first_iid", "nreads", "kmer_len", "tab_bits",
               "slice_bits", "bloom_w", "hash_lib_lo", "hash_lib_hi", "records")


def _hip():
    """The process's HIP runtime (already loaded by torch / libcanu_ovl)."""
    import ctypes
    for name in ("libamdhip64.so.7", "libamdhip64.so.6", "libamdhip64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_int]
            return lib
        except OSError:
            continue
    raise OSError("libamdhip64 not found")


def _agree(ok: bool, dist, dev) -> bool:
    """All ranks' ok flags combined (min), so that a failure on one rank is raised on every
    rank instead of leaving the others waiting in the next collective."""
    if not dist:
        return ok
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _first_failed(ok: bool, dist, dev):
    """The lowest rank whose ok flag is False (None when every rank succeeded): one MIN
    all-reduce of (rank if failed else world), so every rank names the same failing rank."""
    if not dist:
        return None if ok else 0
    import torch
    world = dist.get_world_size()
    t = torch.tensor([world if ok else dist.get_rank()], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    v = int(t.item())
    return None if v >= world else v


def share_index(src, dsts, dist, dev, src_rank: int = 0):
    """Give every rank the index the context `src` built on rank `src_rank`: its buffers
    (ovl_export_index) are copied into torch tensors, broadcast over the process group
    (RCCL over xGMI on the GPUs; dist None: one process, no collective) and imported
    (ovl_import_index) into each context of `dsts` (this rank's contexts holding the same
    reads).  A failure on any rank is raised on all of them.  Returns the bytes moved per
    rank."""
    import torch
    from canu_amd.overlap_in_core import _IndexDesc
    rank = dist.get_rank() if dist else src_rank
    meta = torch.zeros(len(_INDEX_META) + len(_INDEX_PARTS), dtype=torch.int64, device=dev)
    desc, err = None, None
    if rank == src_rank:
        try:
            desc = src.export_index()
            vals = [getattr(desc, f) for f in _INDEX_META] + \
                   [getattr(desc, p + "_bytes") for p in _INDEX_PARTS]
            meta.copy_(torch.tensor(vals, dtype=torch.int64))
        except Exception as e:            # noqa: BLE001 -- re-raised below on every rank
            err = e
    if not _agree(err is None, dist, dev):
        raise RuntimeError(f"share_index: export failed on rank {src_rank}: {err}")
    if dist:
        dist.broadcast(meta, src_rank)
    m = [int(x) for x in meta.tolist()]
    sizes = dict(zip(_INDEX_PARTS, m[len(_INDEX_META):]))
    bufs = {p: torch.empty(max(n, 1), dtype=torch.uint8, device=dev) for p, n in sizes.items()}
    if rank == src_rank:
        try:
            hip = _hip()
            for p in _INDEX_PARTS:
                if sizes[p]:
                    rc = hip.hipMemcpy(bufs[p].data_ptr(), getattr(desc, p), sizes[p], 4)
                    if rc != 0:
                        raise RuntimeError(f"hipMemcpy of the index {p}: error {rc}")
            torch.cuda.synchronize(dev)
        except Exception as e:            # noqa: BLE001
            err = e
    if not _agree(err is None, dist, dev):
        raise RuntimeError(f"share_index: copy failed on rank {src_rank}: {err}")
    if dist:
        for p in _INDEX_PARTS:
            if sizes[p]:
                dist.broadcast(bufs[p], src_rank)
    # the broadcasts run on torch's streams, the import's copies on the library's own: the
    # buffers must be complete before ovl_import_index reads them
    torch.cuda.synchronize(dev)
    d = _IndexDesc()
    for f, v in zip(_INDEX_META, m):
        setattr(d, f, v)
    for p in _INDEX_PARTS:
        setattr(d, p, bufs[p].data_ptr() if sizes[p] else None)
        setattr(d, p + "_bytes", sizes[p])
    try:
        for ctx in dsts:
            ctx.import_index(d)
    except Exception as e:                # noqa: BLE001
        err = e
    torch.cuda.synchronize(dev)
    del bufs
    bad = _first_failed(err is None, dist, dev)
    if bad is not None:
        raise RuntimeError(f"share_index: import failed on rank {bad}"
                           + (f": {err}" if bad == rank else " (its log has the error)"))
    return sum(sizes.values())
