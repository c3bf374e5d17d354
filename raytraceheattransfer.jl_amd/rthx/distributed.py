"""Multi-GPU sharding of the exchange trace.

Emitter rows are independent (the reference already splits them over threads,
parallelRayTracing.jl:81-91) and every ray's random stream is keyed by
(seed, bin, emitter, ray), so a row's counts do not depend on which GPU
traced it.  One process per GPU traces the strided row set
g = rank, rank + W, rank + 2W, ... (strided rather than contiguous so that
surface and volume rows are spread evenly); assembling F is a gather of
disjoint CSR row blocks — there is no reduction, hence no data-path
collective.  ``gather_csr`` uses torch.distributed (gloo on the host) only to
bring the row blocks to rank 0 for the host-side SparseMatrixCSC build.
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


def gather_csr(row_ptr, cols, counts, n: int, group=None):
    """All ranks send their CSR block to rank 0 (torch.distributed object gather).
    Returns the merged CSR on rank 0 and None elsewhere."""
    import torch.distributed as dist

    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    payload = (np.asarray(row_ptr), np.asarray(cols), np.asarray(counts))
    out: List = [None] * world if rank == 0 else None
    dist.gather_object(payload, out, dst=0, group=group)
    if rank != 0:
        return None
    return merge_csr(out, n)
