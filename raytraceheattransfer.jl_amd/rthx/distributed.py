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


# ---------------------------------------------------------------------------
# C5 over W GPUs, row-sharded and pipelined (BASELINE configs[4]).
#
# Every rank traces its rows g = rank, rank + W, ... of EVERY traced band (the
# row stride balances the ranks, which band per GPU cannot: the C5 bands do
# not cost alike), and band i is assembled on its owner rank i mod W: the
# ranks' blocks are gathered there (RCCL over xGMI on an NCCL group) and
# merged in row order on the owner's GPU (rthx_merge_row_shards).  Band i's
# copy-out, gather and merge run on a second host thread and HIP stream while
# band i + 1 traces, so only the last band's assembly is exposed.  The
# reference traces its bins one after another on one host
# (parallelRayTracing.jl:20-42); the counts are the same whoever traces a row
# (counter-based RNG keyed by seed, bin, emitter, ray).
# ---------------------------------------------------------------------------


class TorchBandComm:
    """The pipeline's two collectives on a torch.distributed group: every
    rank's block size (all_gather) and the blocks to the band's owner
    (gather).  Tensors live on the group's device (cuda on NCCL = RCCL,
    cpu on gloo)."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = _device_of(group)

    def all_sizes(self, band: int, n: int) -> List[int]:
        import torch
        import torch.distributed as dist

        out = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in range(self.world)]
        dist.all_gather(out, torch.tensor([n], dtype=torch.int64, device=self.device), group=self.group)
        return [int(x.item()) for x in out]

    def gather(self, band: int, t, dst: int):
        import torch
        import torch.distributed as dist

        out = [torch.empty_like(t) for _ in range(self.world)] if self.rank == dst else None
        dist.gather(t, out, dst=dst, group=self.group)
        return out


class EmulatedBandComm:
    """One GPU standing in for rank `rank` of W (diagnostic: the one-GPU
    projection of tools/bench_c5_bands.py --pipeline, and the GPU tests):
    the other ranks' blocks of the bands this rank owns were traced
    beforehand on this GPU (`peers[band][k]` = (row_off, pairs) tensors of
    rank k), and the gather copies them into fresh buffers on this GPU -- the
    receive's HBM writes, without the xGMI transfer itself."""

    def __init__(self, rank: int, world: int, device: int, peers):
        import torch

        self.rank, self.world = rank, world
        self.device = torch.device("cuda", device)
        self.peers = peers

    @classmethod
    def for_rank(cls, dom, rays: int, rank: int, world: int, device: int = 0, seed: int = 1, nudge: float = None,
                 faithful: bool = False, last_parts: int = 2, order: str = "assembly"):
        """The stand-in for `rank`, its peers' blocks of the bands it owns
        (traced band i is owned by rank i mod W; pieces as band_pieces)
        traced now, on `device`."""
        import torch

        if nudge is None:
            nudge = 10_000 * np.finfo(np.float64).eps
        traced = traced_bands(dom)
        if order == "assembly":
            traced = assembly_order(dom, traced)
        N = dom.flat().n_emitters
        R = rays // N
        tracer = HipShardTracer(dom, device, n_results=1)
        peers = {}
        try:
            for tag, i, _begin, stride, _parts in band_pieces(len(traced), rank, world, last_parts):
                b = traced[i][0]
                if i % world != rank:
                    continue
                h = tag[1] if isinstance(tag, tuple) else 0
                blocks = []
                for k in range(world):
                    if k == rank:
                        blocks.append(None)
                        continue
                    sh = tracer(b - 1, R, nudge, seed, k + h * world, stride, faithful)
                    ro = torch.empty(sh.n_rows + 1, dtype=torch.int64, device=torch.device("cuda", device))
                    pr = torch.empty((2, max(sh.nnz, 1)), dtype=torch.int32, device=ro.device)
                    sh.fill(ro, pr[0], pr[1])
                    sh.done()
                    blocks.append((ro, pr[:, :sh.nnz]))
                peers[tag] = blocks
        finally:
            tracer.close()
        return cls(rank, world, device, peers)

    def all_sizes(self, band: int, n: int) -> List[int]:
        p = self.peers.get(band)
        if p is None:
            return [n] * self.world
        return [n if k == self.rank else int(p[k][1].shape[1]) for k in range(self.world)]

    def gather(self, band: int, t, dst: int):
        import torch

        if self.rank != dst:
            return None
        out = []
        for k in range(self.world):
            if k == self.rank:
                out.append(t)
                continue
            src = self.peers[band][k][0 if t.dtype == torch.int64 else 1]
            o = torch.zeros_like(t)
            if t.dim() == 1:
                o[:src.shape[0]].copy_(src)
            else:
                o[:, :src.shape[1]].copy_(src)
            out.append(o)
        return out


class HipShardTracer:
    """One rank's row shard of a band traced on its GPU (rthx_trace_exchange,
    emitter_begin = rank, emitter_stride = W, counts left on the device).
    Two results alternate: band i + 1 traces into one while band i's counts
    are still being copied out of the other."""

    def __init__(self, dom, device: int = 0, n_results: int = 2):
        import queue

        from ._lib import DeviceResult, device_domain

        self.dd = device_domain(dom, device)
        self.device = device
        self.n = dom.flat().n_emitters
        self._free = queue.Queue()
        self._all = [DeviceResult() for _ in range(n_results)]
        for r in self._all:
            self._free.put(r)

    def __call__(self, bin0: int, R: int, nudge: float, seed: int, begin: int, stride: int, faithful: bool):
        from . import abi
        from ._lib import make_args

        flags = abi.RTHX_FLAG_DEVICE_ONLY | (abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0)
        args, keep = make_args(bin0, R, nudge, seed, begin, self.n, stride, self.device, flags)
        res = self._free.get()  # (waits until the worker has copied a result out)
        try:
            res.trace(self.dd, args)
        except Exception:
            self._free.put(res)
            raise
        del keep
        return _HipShard(res, self._free, begin, stride)

    def close(self):
        for r in self._all:
            r.close()


class _HipShard:
    def __init__(self, res, free, begin: int, stride: int):
        self.res, self._free = res, free
        self.begin, self.stride = begin, stride
        self.info = res.info()
        self.nnz = int(self.info["nnz"])
        self.n_rows = int(self.info["rows_traced"])

    def fill(self, row_off, cols, counts) -> None:
        """The block's CSR into tensors: device to device, or through the
        host for a gloo group's cpu tensors."""
        import ctypes as C

        from ._lib import check, load

        if row_off.device.type == "cpu":
            import torch

            rp, c, v = self.res.csr()  # (over all N rows; the block's are begin, begin + stride, ...)
            lens = np.diff(rp)[self.begin::self.stride]
            row_off[0] = 0
            row_off[1:len(lens) + 1] = torch.from_numpy(np.cumsum(lens))
            cols[:self.nnz] = torch.from_numpy(c[:self.nnz])
            counts[:self.nnz] = torch.from_numpy(v[:self.nnz].view(np.int32))
            return
        check(load().rthx_result_copy_csr_device(self.res.handle, 0, C.c_void_p(row_off.data_ptr()),
                                                 C.c_void_p(cols.data_ptr()), C.c_void_p(counts.data_ptr())))

    def done(self) -> None:
        self._free.put(self.res)


def merge_row_shards_device(row_offs, cols, counts, n_rows: int, sizes=None, stream=None):
    """Merge W strided row blocks (block k: rows k, k + W, ...; local row
    offsets) that lie on one GPU into one CSR in row order with the HIP
    kernels of rthx_merge_row_shards.  sizes: the blocks' entry counts when
    known (else read from their offsets).  Returns (row_ptr int64
    [n_rows + 1], cols int32, counts int32 holding the uint32 bits),
    enqueued on `stream` (default: torch's current stream)."""
    import ctypes as C

    import torch

    from ._lib import check, load

    W = len(row_offs)
    dev = row_offs[0].device
    if sizes is None:
        sizes = []
        for k in range(W):
            n_k = len(range(k, n_rows, W))
            sizes.append(int(row_offs[k][n_k].item()) - int(row_offs[k][0].item()))
    total = int(sum(sizes))
    row_ptr = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
    out_c = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    out_n = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    arr = C.c_void_p * W
    ro = arr(*[C.c_void_p(t.data_ptr()) for t in row_offs])
    cc = arr(*[C.c_void_p(t.data_ptr()) for t in cols])
    nn = arr(*[C.c_void_p(t.data_ptr()) for t in counts])
    st = stream if stream is not None else torch.cuda.current_stream(dev)
    check(load().rthx_merge_row_shards(dev.index, W, n_rows, ro, cc, nn, C.c_void_p(row_ptr.data_ptr()),
                                       C.c_void_p(out_c.data_ptr()), C.c_void_p(out_n.data_ptr()),
                                       C.c_void_p(st.cuda_stream)))
    return row_ptr, out_c[:total], out_n[:total]


def merge_row_shards_host(row_offs, cols, counts, n_rows: int):
    """The same merge on the host (numpy; a gloo group's blocks)."""
    W = len(row_offs)
    lens = np.zeros(n_rows, dtype=np.int64)
    for k in range(W):
        n_k = len(range(k, n_rows, W))
        ro = np.asarray(row_offs[k][:n_k + 1], dtype=np.int64)
        lens[k::W] = np.diff(ro)
    row_ptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.cumsum(lens, out=row_ptr[1:])
    total = int(row_ptr[-1])
    out_c = np.zeros(total, dtype=np.int32)
    out_n = np.zeros(total, dtype=np.uint32)
    for k in range(W):
        rows = np.arange(k, n_rows, W)
        ro = np.asarray(row_offs[k][:len(rows) + 1], dtype=np.int64)
        lk = np.diff(ro)
        tot = int(lk.sum())
        if tot == 0:
            continue
        dst = np.repeat(row_ptr[rows] - (ro[:-1] - ro[0]), lk) + np.arange(tot)
        out_c[dst] = np.asarray(cols[k])[ro[0]:ro[0] + tot]
        out_n[dst] = np.asarray(counts[k]).view(np.uint32)[ro[0]:ro[0] + tot]
    return row_ptr, out_c, out_n


def _assemble_piece(comm, tag, shard, owner: int, n_rows: int, parts: int, held: dict, stream):
    """One traced piece of a band -- the whole band (parts = 1), or piece h
    of `parts` (rows rank + h W, stride parts W) -- copied out of this
    rank's trace and gathered to the band's owner (runs on the pipeline's
    second thread).  The owner merges once the band's last piece has
    arrived: block h W + k of the merge is rank k's piece h, the rows
    congruent to h W + k modulo parts W.  Returns the owner's (row_ptr,
    cols, counts) after the last piece, None otherwise."""
    import torch

    W = comm.world
    band, h = tag if isinstance(tag, tuple) else (tag, 0)
    n_sh = parts * W
    sizes = comm.all_sizes(tag, shard.nnz)
    cap = max(max(sizes), 1)
    nmax = (n_rows + n_sh - 1) // n_sh
    dev = comm.device
    ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
    with ctx:
        row_off = torch.zeros(nmax + 1, dtype=torch.int64, device=dev)
        pairs = torch.zeros((2, cap), dtype=torch.int32, device=dev)
        if stream is not None:
            stream.synchronize()  # (the buffers exist before the library's stream writes them)
        shard.fill(row_off, pairs[0], pairs[1])
        shard.done()
        ros = comm.gather(tag, row_off, owner)
        prs = comm.gather(tag, pairs, owner)
        if ros is None:
            if stream is not None:
                stream.synchronize()  # (the gather has read this rank's buffers)
            return None
        got = held.setdefault(band, {})
        got[h] = (ros, prs, sizes)
        if len(got) < parts:
            return None
        del held[band]
        blocks = [(got[hh][0][k], got[hh][1][k], got[hh][2][k]) for hh in range(parts) for k in range(W)]
        if dev.type == "cuda":
            out = merge_row_shards_device([x[0] for x in blocks], [x[1][0] for x in blocks],
                                          [x[1][1] for x in blocks], n_rows, [x[2] for x in blocks], stream)
            stream.synchronize()
            return out
        return merge_row_shards_host([x[0].numpy() for x in blocks], [x[1][0].numpy() for x in blocks],
                                     [x[1][1].numpy() for x in blocks], n_rows)


def assembly_order(dom, traced):
    """The traced bands in the pipeline's order: the reference's
    (traced_bands), except that the band with the smallest optical
    thickness (sum over fine cells of beta x area) goes last.  Only the last
    band's gather and merge follow the last trace, and a transparent band's
    rays end on few absorbers -- the walls -- so its count matrix is the
    smallest to gather (C5 at 1e9 rays: 33 M nonzeros against 221 M for an
    opaque band).  Any order gives the same bands; every rank computes the
    same one."""
    flat = dom.flat()
    nf = len(flat.fine_volume)
    beta = np.asarray(flat.beta).reshape(-1, nf)
    area = np.abs(np.asarray(flat.fine_volume))
    tau = [float(np.dot(beta[b - 1], area)) for b, _ in traced]
    k = int(np.argmin(tau))
    return [t for i, t in enumerate(traced) if i != k] + [traced[k]]


def band_pieces(n_traced: int, rank: int, world: int, last_parts: int = 1):
    """The traces one rank runs, in order: (tag, traced-band index, emitter
    begin, stride, parts).  Every band whole (rows rank, rank + W, ...) but
    the last, which is traced in last_parts pieces (rows rank + h W,
    stride last_parts W) so that its first pieces' gathers run while its
    last one traces."""
    out = []
    for i in range(n_traced):
        P = last_parts if i == n_traced - 1 else 1
        if P == 1:
            out.append((i, i, rank, world, 1))
        else:
            out.extend(((i, h), i, rank + h * world, P * world, P) for h in range(P))
    return out


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def trace_bands_row_sharded(dom, rays: int, group=None, seed: int = 1, nudge: float = None, device: int = 0,
                            faithful: bool = False, overlap: bool = True, tracer=None, comm=None,
                            last_parts: int = 2, order: str = "assembly"):
    """C5 (:spectral_variable) over W ranks, row-sharded and pipelined (see the
    section comment above).  rays: per band, as mesh() (R = rays // N rays
    per emitter).  Every rank traces its rows of every traced band
    (traced_bands order); traced band i is assembled on rank i mod W.

    Returns (owned, info): owned maps each traced bin this rank owns
    (1-based, as traced_bands) to its count matrix in row order (row_ptr,
    cols, counts) -- tensors on the rank's GPU on an NCCL group (counts:
    int32 holding the uint32 bits), numpy on gloo -- and info holds each
    band's trace info and the host-clock timeline (trace and assembly
    intervals, seconds from the start; wall_s: from the first trace to the
    last assembly, call_s: the whole call).  overlap=False assembles each
    band before the next traces (the sequential form, for comparison).
    last_parts: the last band is traced in that many pieces, so that only
    its last piece's gather and the merge follow the last trace
    (band_pieces).  order: "assembly" (assembly_order: the most transparent
    band last) or "reference" (traced_bands as is); traced band i of the
    order is owned by rank i mod W.
    tracer / comm: stand-ins for tests and the one-GPU emulation
    (tools/bench_c5_bands.py); the product uses HipShardTracer and
    TorchBandComm."""
    import threading
    import time
    from concurrent.futures import ThreadPoolExecutor

    comm = comm or TorchBandComm(group)
    W, rank = comm.world, comm.rank
    if nudge is None:
        nudge = 10_000 * np.finfo(np.float64).eps
    traced = traced_bands(dom)
    if order == "assembly":
        traced = assembly_order(dom, traced)
    N = dom.flat().n_emitters
    R = rays // N
    own_tracer = tracer is None
    tracer = tracer or HipShardTracer(dom, device)
    stream = None
    if comm.device.type == "cuda":
        import torch

        stream = torch.cuda.Stream(device=comm.device)
    t0 = time.perf_counter()
    timeline = []
    lock = threading.Lock()

    held = {}  # (owner) pieces of a band gathered so far

    def assemble(tag, i, b, shard, parts):
        import torch

        if comm.device.type == "cuda":
            torch.cuda.set_device(comm.device)
        ta = time.perf_counter() - t0
        out = _assemble_piece(comm, tag, shard, i % W, N, parts, held, stream)
        with lock:
            timeline.append({"band": b, "what": "assemble", "owner": i % W, "start_s": ta,
                             "end_s": time.perf_counter() - t0, "piece": tag[1] if isinstance(tag, tuple) else None})
        return out

    owned, infos, futs = {}, [], []
    ex = ThreadPoolExecutor(max_workers=1) if overlap else None
    try:
        for tag, i, begin, stride, parts in band_pieces(len(traced), rank, W, last_parts):
            b = traced[i][0]
            ts = time.perf_counter() - t0
            shard = tracer(b - 1, R, nudge, seed, begin, stride, faithful)
            te = time.perf_counter() - t0
            inf = dict(shard.info, bin=b)
            infos.append(inf)
            with lock:
                timeline.append({"band": b, "what": "trace", "start_s": ts, "end_s": te,
                                 "kernel_ms": inf.get("trace_ms"), "pack_ms": inf.get("pack_ms"),
                                 "piece": tag[1] if isinstance(tag, tuple) else None})
            if ex is not None:
                futs.append((b, ex.submit(assemble, tag, i, b, shard, parts)))
            else:
                out = assemble(tag, i, b, shard, parts)
                if out is not None:
                    owned[b] = out
        for b, f in futs:
            out = f.result()
            if out is not None:
                owned[b] = out
    finally:
        if ex is not None:
            ex.shutdown(wait=True)
        if own_tracer:
            tracer.close()
    total = time.perf_counter() - t0
    timeline.sort(key=lambda e: (e["start_s"], e["what"]))
    wall = max(e["end_s"] for e in timeline) - min(e["start_s"] for e in timeline) if timeline else 0.0
    return owned, {"world": W, "rank": rank, "rays_per_emitter": R, "traces": infos, "timeline": timeline,
                   "wall_s": wall, "call_s": total, "last_parts": last_parts,
                   "owner": {b: i % W for i, (b, _) in enumerate(traced)}}
