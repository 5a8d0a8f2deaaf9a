"""Multi-process path on CPU (gloo, world_size 2): the setup all-gather of the read store
that bench.py does over RCCL, and independent query shards whose union is the whole job."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle
    from canu_amd.dist import gather_read_store, query_shards
    from canu_amd.synth import ReadSet, random_genome, synth_reads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, L, G = 50, 1800, 9000
    genome = random_genome(np.random.default_rng(5), G)
    lo, hi = n * rank // world, n * (rank + 1) // world
    part = synth_reads(n, L, G, 0.02, seed=5, genome=genome, read_range=(lo, hi))
    bases, lengths = gather_read_store(torch.from_numpy(part.bases), part.lengths, dist,
                                       torch.device("cpu"))
    offsets = np.zeros(n, dtype=np.uint64)
    offsets[1:] = np.cumsum(lengths[:-1], dtype=np.uint64)
    rs = ReadSet(bases=bases.numpy(), offsets=offsets, lengths=lengths)
    p = oracle.default_params(kmer_len=22, max_erate=0.06, min_olap_len=200)
    q_lo, q_hi = query_shards(n, world)[rank]
    # each rank indexes only reads q_lo..n: its queries' targets all have larger IDs
    mine = oracle.run_oracle(rs, p, hash_range=(q_lo, n), ref_range=(q_lo, q_hi))
    counts = [None] * world
    dist.all_gather_object(counts, mine.tobytes())
    if rank == 0:
        whole = synth_reads(n, L, G, 0.02, seed=5, genome=genome)
        ok_store = (np.array_equal(rs.bases, whole.bases) and
                    np.array_equal(rs.lengths, whole.lengths))
        union = np.concatenate([np.frombuffer(b, dtype=oracle.RECORD_DTYPE) for b in counts])
        ok_union = np.array_equal(oracle.sort_records(union), oracle.run_oracle(whole, p))
        q.put((ok_store, ok_union, len(union)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok_store, ok_union, n = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok_store and ok_union and n > 0


def _mhap_worker(rank, world, port, q):
    """MHAP's multi-GPU split on CPU: each rank sketches its slice of the reads, the sketch
    rows are all-gathered (bench_mhap.py does this over RCCL), each rank compares its own
    query shard; the gathered rows equal the whole job's and the shards union to it."""
    import torch
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    import mhap_jar as M
    from canu_amd.dist import all_gather_rows, query_shards, read_slices
    from canu_amd.synth import ReadSet, synth_reads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, L = 41, 3000
    rs = synth_reads(n, L, n * L // 12, 0.04, seed=9)
    p = M.default_params(num_hashes=64, ordered_sketch=600, min_olap=300)
    lo, hi = read_slices(n, world)[rank]
    part = ReadSet(bases=rs.bases, offsets=rs.offsets[lo:hi], lengths=rs.lengths[lo:hi])
    # the library's row layout: [read][strand][H] / [read][strand][S] / [read][strand]
    rows = M.sketch_rows(part, p)
    full = [all_gather_rows(torch.from_numpy(r.reshape(hi - lo, -1).view(np.int32)), n,
                            dist).numpy() for r in rows]
    q_lo, q_hi = query_shards(n, world)[rank]
    recs = M.run(rs, p, q_range=(q_lo - 1, q_hi))
    got = [None] * world
    dist.all_gather_object(got, recs.tobytes())
    if rank == 0:
        whole = M.run(rs, p)
        union = np.concatenate([np.frombuffer(b, dtype=M.MHAP_DTYPE) for b in got])
        union = union[np.lexsort((union["o"], union["b"], union["a"]))]
        want = [r.reshape(n, -1).view(np.int32) for r in M.sketch_rows(rs, p)]
        q.put((all(np.array_equal(a, b) for a, b in zip(full, want)),
               np.array_equal(union, whole), len(whole)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_mhap_sketch_gather_and_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mhap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok_rows, ok_union, n = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok_rows and ok_union and n > 0


def _prefix_worker(rank, world, port, q):
    """configs[4]'s setup exchange (dist.gather_read_prefix): rank r gets reads 1..need_r
    only -- the reads its `-h lo-hi -r 1-hi` job touches -- point to point from the ranks
    that generated them, and holds nothing more; and dist._first_failed names the same
    failing rank on every rank."""
    import torch
    import torch.distributed as dist
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from canu_amd.dist import _first_failed, gather_read_prefix, read_slices
    from canu_amd.synth import random_genome, synth_reads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, L, G = 61, 900, 8000
    genome = random_genome(np.random.default_rng(7), G)
    lo, hi = read_slices(n, world)[rank]
    part = synth_reads(n, L, G, 0.02, seed=7, genome=genome, read_range=(lo, hi),
                       len_jitter=0.3)
    # a hash-block plan's needs: increasing with the rank, the last rank the whole store
    needs = [int(n * (r + 1) ** 2 // world ** 2) for r in range(world)]
    needs[0] = max(needs[0], 1)
    bases, lengths = gather_read_prefix(torch.from_numpy(part.bases), part.lengths,
                                        needs[rank], dist, torch.device("cpu"))
    whole = synth_reads(n, L, G, 0.02, seed=7, genome=genome, len_jitter=0.3)
    m = needs[rank]
    ok = (lengths.shape[0] == m and np.array_equal(lengths, whole.lengths[:m]) and
          bases.numel() == int(whole.lengths[:m].sum()) and
          np.array_equal(bases.numpy(), whole.bases[:bases.numel()]))
    fail_rank = world - 1
    named = _first_failed(rank != fail_rank, dist, torch.device("cpu"))
    none = _first_failed(True, dist, torch.device("cpu"))
    res = [None] * world
    dist.all_gather_object(res, (ok, named, none))
    if rank == 0:
        q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_read_prefix_per_rank(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prefix_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for ok, named, none in res:
        assert ok
        assert named == world - 1 and none is None
