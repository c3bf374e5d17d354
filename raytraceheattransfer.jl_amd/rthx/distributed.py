"""Multi-GPU sharding of the exchange trace.

Emitter rows are independent (the reference already splits them over threads,
parallelRayTracing.jl:81-91) and every ray's random stream is keyed by
(seed, bin, emitter, ray), so a row's counts do not depend on which GPU
traced it.  One process per GPU traces the strided row set
g = rank, rank + W, rank + 2W, ... (strided rather than contiguous so that
surface and volume rows are spread evenly); assembling F is a gather of
disjoint CSR row blocks — there is no reduction, hence no data-path
collective.  ``gather_csr`` brings the row blocks to one rank (or all) when
the caller wants the whole F: tensor all-reduce / all-gather, over RCCL and
xGMI on an NCCL group, over gloo on the host otherwise.  Inside one process,
rthx_multi_trace_exchange splits rows over several devices instead.

Spectral domains whose bands vary in space (:spectral_variable, BASELINE
config C5: every band traced alone, parallelRayTracing.jl:20-42) also shard
by band: each rank (or each device of one process,
rthx.exchange.parallel_ray_tracing with band devices) traces whole bands,
``bands_of`` picking its share of the traced bands.  Bands are independent,
so again there is no collective on the data path; ``broadcast_csr`` hands a
band's CSR to the other ranks when they want it.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard(rank: int, world: int) -> Tuple[int, int]:
    """(emitter_begin, emitter_stride) of `rank`'s rows."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return rank, world


def rows_of(rank: int, world: int, n_emitters: int) -> np.ndarray:
    b, s = shard(rank, world)
    return np.arange(b, n_emitters, s, dtype=np.int64)


def merge_csr(pieces: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]], n: int):
    """Merge CSR blocks with disjoint row sets (each over all n rows) into one CSR."""
    nnz_per_row = np.zeros(n, dtype=np.int64)
    for rp, _c, _v in pieces:
        nnz_per_row += np.diff(rp)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(nnz_per_row, out=row_ptr[1:])
    nnz = int(row_ptr[-1])
    cols = np.zeros(nnz, dtype=np.int32)
    counts = np.zeros(nnz, dtype=np.uint32)
    for rp, c, v in pieces:
        lens = np.diff(rp)
        rows = np.nonzero(lens)[0]
        if rows.size == 0:
            continue
        # destination ranges for this piece's non-empty rows
        dst = np.concatenate([np.arange(row_ptr[r], row_ptr[r] + lens[r]) for r in rows])
        src = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows])
        if np.any(nnz_per_row[rows] != lens[rows]):
            raise ValueError("row blocks overlap")
        cols[dst] = c[src]
        counts[dst] = v[src]
    return row_ptr, cols, counts


def _place(pieces_rows, pieces, lens_global, row_ptr, nnz):
    """Scatter CSR pieces (each: its rows ascending, their entries in row
    order) into the global arrays."""
    cols = np.zeros(nnz, dtype=np.int32)
    counts = np.zeros(nnz, dtype=np.uint32)
    for rows, (c, v) in zip(pieces_rows, pieces):
        lens = lens_global[rows]
        tot = int(lens.sum())
        if tot == 0:
            continue
        src_start = np.concatenate(([0], np.cumsum(lens)[:-1]))
        dst = np.repeat(row_ptr[rows] - src_start, lens) + np.arange(tot)
        cols[dst] = c[:tot]
        counts[dst] = v[:tot]
    return cols, counts


def gather_csr(row_ptr, cols, counts, n: int, group=None, dst: int = 0):
    """Bring every rank's CSR block (disjoint row sets, each over all n rows)
    to rank `dst` (dst = -1: to every rank) with tensor collectives: one
    all-reduce of the row lengths and owners, one all-gather of the padded
    (col, count) pairs.  On an NCCL (= RCCL on ROCm) group the tensors travel
    over xGMI from device memory; on gloo through the host.  Returns the
    merged CSR (row_ptr, cols, counts) where requested, else None."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    rp = np.asarray(row_ptr, dtype=np.int64)
    lens = np.diff(rp)
    nnz_local = int(rp[-1])
    mine = np.zeros(n, dtype=np.int64)
    mine[lens > 0] = rank + 1
    meta = torch.from_numpy(np.concatenate([lens, mine, [nnz_local]])).to(dev)
    # lengths and owners (disjoint rows: the sums are the values), and the
    # largest block for the padding
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, meta[-1:].clone(), group=group)
    meta = meta[:-1]
    dist.all_reduce(meta, group=group)
    meta = meta.cpu().numpy()
    lens_g, owner = meta[:n], meta[n:]
    nnz_k = [int(x.item()) for x in sizes]
    cap = max(max(nnz_k), 1)
    buf = np.zeros((2, cap), dtype=np.int64)
    buf[0, :nnz_local] = np.asarray(cols, dtype=np.int64)[:nnz_local]
    buf[1, :nnz_local] = np.asarray(counts, dtype=np.int64)[:nnz_local]
    t = torch.from_numpy(buf).to(dev)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    if dst >= 0 and rank != dst:
        return None
    g_rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens_g, out=g_rp[1:])
    pieces = [(o[0].cpu().numpy(), o[1].cpu().numpy()) for o in out]
    rows = [np.nonzero(owner == k + 1)[0] for k in range(world)]
    c, v = _place(rows, pieces, lens_g, g_rp, int(g_rp[-1]))
    return g_rp, c, v


def traced_bands(dom) -> List[Tuple[int, List[int]]]:
    """The traces a :spectral_variable mesh() runs, in the reference's order
    (parallelRayTracing.jl:20-42): (traced bin, bins that share its F), 1-based
    -- every non-uniform bin alone, then one trace per group of uniform bins
    with equal beta (group_uniform_bins)."""
    from .exchange import group_uniform_bins

    groups, _reps, nonuniform = group_uniform_bins(dom.uniform_across_bin)
    return [(b, [b]) for b in nonuniform] + [(g[0], list(g)) for g in groups]


def bands_of(rank: int, world: int, traced: Sequence[Tuple[int, List[int]]]):
    """`rank`'s share of the traced bands (every world-th, in trace order)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return [t for k, t in enumerate(traced) if k % world == rank]


def broadcast_csr(row_ptr, cols, counts, n: int, src: int, group=None):
    """Rank `src`'s CSR (n rows) on every rank: the sizes, then the arrays,
    as tensor broadcasts (over RCCL / xGMI on an NCCL group, gloo on the host).
    Non-source ranks pass None for the arrays."""
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    rank = dist.get_rank(group)
    nnz = torch.tensor([int(row_ptr[-1]) if rank == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(nnz, src, group=group)
    m = int(nnz.item())
    if rank == src:
        buf = torch.from_numpy(np.concatenate([np.asarray(row_ptr, dtype=np.int64),
                                               np.asarray(cols, dtype=np.int64)[:m],
                                               np.asarray(counts, dtype=np.int64)[:m]])).to(dev)
    else:
        buf = torch.empty(n + 1 + 2 * m, dtype=torch.int64, device=dev)
    dist.broadcast(buf, src, group=group)
    b = buf.cpu().numpy()
    return b[:n + 1], b[n + 1:n + 1 + m].astype(np.int32), b[n + 1 + m:].astype(np.uint32)
