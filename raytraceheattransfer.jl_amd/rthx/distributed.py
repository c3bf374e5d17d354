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


def _device_of(group):
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _pairs_tensor(cols, counts, dev):
    """(cols, counts) as one int32 [2, nnz] tensor on `dev`: the uint32
    counts travel bit for bit as int32 (8 bytes per nonzero)."""
    import torch

    if isinstance(cols, torch.Tensor):
        return torch.stack([cols.to(dev, torch.int32), counts.to(dev).view(torch.int32)
                            if counts.dtype == torch.int32 else counts.to(dev, torch.int32)])
    c = np.ascontiguousarray(cols, dtype=np.int32)
    v = np.ascontiguousarray(counts, dtype=np.uint32).view(np.int32)
    return torch.from_numpy(np.stack([c, v])).to(dev)


def _gather_blocks(rows, lens, pairs, n: int, group, dst: int, as_tensors: bool):
    """The gather behind gather_csr / gather_result.  rows: this rank's
    traced rows (global ids, ascending), lens: their entry counts, pairs: the
    int32 [2, nnz] (col, count) tensor of those rows in row order (on the
    group's device)."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    dev = pairs.device
    rows = torch.as_tensor(rows, dtype=torch.int64, device=dev)
    lens = torch.as_tensor(lens, dtype=torch.int64, device=dev)
    nnz_local = int(pairs.shape[1])
    # row lengths and owners over all n rows (disjoint rows: the sums are
    # the values), to dst only when dst >= 0
    meta = torch.zeros(2 * n, dtype=torch.int64, device=dev)
    meta[rows] = lens
    meta[n + rows] = rank + 1
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([nnz_local], dtype=torch.int64, device=dev), group=group)
    cap = max(max(int(x.item()) for x in sizes), 1)
    buf = torch.zeros((2, cap), dtype=torch.int32, device=dev)
    buf[:, :nnz_local] = pairs
    if dst >= 0:
        dist.reduce(meta, dst, group=group)
        out = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
        dist.gather(buf, out, dst=dst, group=group)
        if rank != dst:
            return None
    else:
        dist.all_reduce(meta, group=group)
        out = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(out, buf, group=group)
    lens_g, owner = meta[:n], meta[n:]
    g_rp = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens_g, 0, out=g_rp[1:])
    total = int(g_rp[-1].item())
    cols = torch.zeros(total, dtype=torch.int32, device=dev)
    counts = torch.zeros(total, dtype=torch.int32, device=dev)
    for k in range(world):
        rk = torch.nonzero(owner == k + 1).flatten()
        lk = lens_g[rk]
        tot = int(lk.sum().item()) if rk.numel() else 0
        if tot == 0:
            continue
        start = torch.cumsum(lk, 0) - lk  # each row's first entry in rank k's block
        idx = torch.repeat_interleave(g_rp[rk] - start, lk) + torch.arange(tot, device=dev)
        cols[idx] = out[k][0, :tot]
        counts[idx] = out[k][1, :tot]
    if as_tensors:
        return g_rp, cols, counts
    return g_rp.cpu().numpy(), cols.cpu().numpy(), counts.cpu().numpy().view(np.uint32)


def gather_csr(row_ptr, cols, counts, n: int, group=None, dst: int = 0, as_tensors: bool = False):
    """Bring every rank's CSR block (disjoint row sets, each over all n rows)
    to rank `dst` (dst = -1: to every rank) with tensor collectives: the
    (col, count) pairs as int32 (8 bytes per nonzero) gathered to dst alone
    (all-gathered only for dst = -1), the row lengths and owners reduced
    there.  On an NCCL (= RCCL on ROCm) group the tensors travel over xGMI
    from device memory; on gloo through the host.  Returns the merged CSR
    (row_ptr, cols, counts) on the receiving ranks (numpy, or tensors on the
    group's device with as_tensors: counts are then int32 tensors holding
    the uint32 bits, so counts >= 2^31 read negative until viewed as
    uint32), None elsewhere."""
    dev = _device_of(group)
    rp = np.asarray(row_ptr, dtype=np.int64)
    lens = np.diff(rp)
    rows = np.nonzero(lens)[0]
    nnz_local = int(rp[-1])
    pairs = _pairs_tensor(np.asarray(cols)[:nnz_local], np.asarray(counts)[:nnz_local], dev)
    return _gather_blocks(rows, lens[rows], pairs, n, group, dst, as_tensors)


def gather_result(res, n: int, group=None, dst: int = 0, as_tensors: bool = False):
    """gather_csr of a traced rthx result (rthx._lib.DeviceResult).  On an NCCL
    group the counts never leave device memory before the collective: each
    block of the result (one per device of a MultiDeviceDomain trace, rows
    emitter_begin + k * emitter_stride) is copied device to device
    (rthx_result_copy_csr_device) and onto this rank's device, and the
    blocks' rows are put in ascending order before the tensors go to RCCL.
    On gloo the host CSR is gathered.  With as_tensors the counts come back
    as int32 tensors holding the uint32 bits (counts >= 2^31 read negative:
    ``counts.view(torch.int32)`` reinterpreted, ``.cpu().numpy().view(np.uint32)``
    restores them); the numpy form is uint32."""
    import torch

    dev = _device_of(group)
    if dev.type == "cuda":
        n_parts = int(res.device_csr(0)["n_parts"])
        rows_l, lens_l, pairs_l = [], [], []
        for part in range(n_parts):
            row_off, pairs, d = res.torch_csr(part)
            row_off, pairs = row_off.to(dev), pairs.to(dev)
            rows_l.append(d["emitter_begin"] + d["emitter_stride"]
                          * torch.arange(d["n_rows"], dtype=torch.int64, device=dev))
            lens_l.append(row_off[1:] - row_off[:-1])
            pairs_l.append(pairs)
        rows, lens, pairs = torch.cat(rows_l), torch.cat(lens_l), torch.cat(pairs_l, dim=1)
        if n_parts > 1:  # interleaved blocks: entries regrouped by ascending row
            order = torch.argsort(rows)
            start = torch.cumsum(lens, 0) - lens
            lo = lens[order]
            tot = int(lo.sum().item())
            first = torch.cumsum(lo, 0) - lo
            idx = torch.repeat_interleave(start[order] - first, lo) + torch.arange(tot, device=dev)
            rows, lens, pairs = rows[order], lo, pairs[:, idx]
        keep = lens > 0
        return _gather_blocks(rows[keep], lens[keep], pairs, n, group, dst, as_tensors)
    rp, c, v = res.csr()
    return gather_csr(rp, c, v, n, group=group, dst=dst, as_tensors=as_tensors)


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
    """Rank `src`'s CSR (n rows) on every rank: the sizes, the row pointers
    (int64) and the (col, count) pairs (int32, 8 bytes per nonzero) as tensor
    broadcasts (over RCCL / xGMI on an NCCL group, gloo on the host).
    Non-source ranks pass None for the arrays."""
    import torch
    import torch.distributed as dist

    dev = _device_of(group)
    rank = dist.get_rank(group)
    nnz = torch.tensor([int(row_ptr[-1]) if rank == src else 0], dtype=torch.int64, device=dev)
    dist.broadcast(nnz, src, group=group)
    m = int(nnz.item())
    if rank == src:
        rp = torch.from_numpy(np.ascontiguousarray(row_ptr, dtype=np.int64)).to(dev)
        pairs = _pairs_tensor(np.asarray(cols)[:m], np.asarray(counts)[:m], dev)
    else:
        rp = torch.empty(n + 1, dtype=torch.int64, device=dev)
        pairs = torch.empty((2, m), dtype=torch.int32, device=dev)
    dist.broadcast(rp, src, group=group)
    dist.broadcast(pairs, src, group=group)
    p = pairs.cpu().numpy()
    return rp.cpu().numpy(), p[0].copy(), p[1].view(np.uint32).copy()
