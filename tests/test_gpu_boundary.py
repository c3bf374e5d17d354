"""The C-ABI boundary beyond one plain trace, on the GPU: the multi-device
trace (rthx_multi_trace_exchange), F_raw formed on the device
(rthx_result_copy_F), DMA into page-locked caller memory, the look-back's
fallback to the staging path, and trace -> smooth -> solve without F_raw
leaving the device.

Counts are compared exactly (every row is a pure function of (seed, bin,
emitter, ray)); F values to 1e-15 relative (one division each); smoothing
results to 1e-12 (iterative fp64 with different reduction orders).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import helpers as H
from oracle import oracle

pytestmark = pytest.mark.gpu


def _args(hip, flat, R, seed=1, bin0=0, begin=0, end=None, stride=1, rec=None, flags=0):
    return hip.make_args(bin0, R, H.NUDGE, seed, begin, flat.n_emitters if end is None else end, stride,
                         flags=flags, record_ids=rec)


def _trace(hip, dd, args, pinned=None):
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        info = res.info()
        rp, cols, cnt = res.csr(pinned)
        out = (rp.copy(), cols.copy(), cnt.copy(), info)
    finally:
        res.close()
    return out


@pytest.mark.parametrize("case", ["square", "greenhouse", "wedges"])
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_multi_device_equals_one_device(hip, case, devices):
    """Rows split over several device slots (contiguous blocks on the
    single-polygon square, interleaved rows on the multi-polygon greenhouse
    and wedges) give the one-device counts bit for bit.  On a one-GPU box the
    slots are concurrent streams of device 0."""
    dom = {"square": lambda: H.square_domain(31), "greenhouse": lambda: H.greenhouse_domain(12, 21, 3, 8),
           "wedges": lambda: H.wedge_domain(16, 4)}[case]()
    flat = dom.flat()
    for bin0 in ((0, 5) if case == "greenhouse" else (0,)):
        args, _k = _args(hip, flat, 3000, seed=21, bin0=bin0)
        dd = hip.DeviceDomain(flat, 0)
        one = _trace(hip, dd, args)
        dd.close()
        md = hip.MultiDeviceDomain(flat, devices)
        multi = _trace(hip, md, args)
        md.close()
        assert multi[3]["n_devices"] == len(devices)
        for a, b in zip(one[:3], multi[:3]):
            assert np.array_equal(a, b)
        for k in ("nnz", "lost_total", "lost_max_row", "rays_traced", "rows_traced"):
            assert one[3][k] == multi[3][k], k


def test_multi_device_shard_and_recorder(hip):
    """A strided row subset and recorded emitters through the multi-device
    trace equal the oracle (recorded rays in emitter order)."""
    dom = H.wedge_domain(8, 3)
    flat = dom.flat()
    ids = [0, 5, 17, flat.n_emitters - 1]
    args, _k = _args(hip, flat, 700, seed=7, rec=ids)
    md = hip.MultiDeviceDomain(flat, [0, 0, 0])
    res = hip.DeviceResult()
    try:
        res.trace(md, args)
        rp, cols, cnt = res.csr()
        o, e, g = res.rays()
    finally:
        res.close()
        md.close()
    orp, ocols, ocnt, oinfo, (oo, oe, og) = oracle.trace_exchange(flat, args, 16)
    assert np.array_equal(rp, orp) and np.array_equal(cols, ocols) and np.array_equal(cnt, ocnt)
    order = np.lexsort((np.arange(len(og)), og))
    assert np.array_equal(g, og[order])
    assert np.allclose(o, oo[order], rtol=0, atol=1e-12)
    args, _k = _args(hip, flat, 900, seed=8, begin=2, stride=5)
    md = hip.MultiDeviceDomain(flat, [0, 0])
    got = _trace(hip, md, args)
    md.close()
    ref = oracle.trace_exchange(flat, args, 16)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2])


def test_recorder_on_single_polygon_domain(hip):
    """Recording on a one-polygon domain runs the staging kernels (never the
    direct-CSR look-back): counts and rays equal the oracle."""
    dom = H.square_domain(9)
    flat = dom.flat()
    ids = [0, 3, flat.n_emitters - 1]
    args, _k = _args(hip, flat, 1500, seed=4, rec=ids)
    dd = hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        rp, cols, cnt = res.csr()
        o, e, g = res.rays()
    finally:
        res.close()
        dd.close()
    orp, ocols, ocnt, oinfo, (oo, oe, og) = oracle.trace_exchange(flat, args, 16)
    assert np.array_equal(rp, orp) and np.array_equal(cols, ocols) and np.array_equal(cnt, ocnt)
    order = np.lexsort((np.arange(len(og)), og))
    assert np.array_equal(g, og[order])
    assert np.allclose(e, oe[order], rtol=0, atol=1e-9)


def test_copy_F_is_normalised_counts(hip):
    """rthx_result_copy_F: F_raw = count / tallied per row (the reference's
    count / R followed by row_normalize!), same pattern as the counts; rows
    sum to 1; also through the multi-device result and into pinned arrays."""
    dom = H.wedge_domain(8, 3)  # open spokes: some rays lost, so tallied < R in places
    flat = dom.flat()
    args, _k = _args(hip, flat, 2500, seed=9)
    for kind in ("one", "multi"):
        dd = hip.DeviceDomain(flat, 0) if kind == "one" else hip.MultiDeviceDomain(flat, [0, 0])
        pin = hip.PinnedArrays()
        res = hip.DeviceResult()
        try:
            res.trace(dd, args)
            rp, cols, cnt = [x.copy() for x in res.csr()]
            frp, fcols, vals = [x.copy() for x in res.F(pin)]
        finally:
            res.close()
            dd.close()
            pin.close()
        assert np.array_equal(rp, frp) and np.array_equal(cols, fcols)
        tallied = np.add.reduceat(cnt.astype(np.int64), rp[:-1][np.diff(rp) > 0])
        want = cnt / np.repeat(tallied, np.diff(rp)[np.diff(rp) > 0])
        np.testing.assert_allclose(vals, want, rtol=1e-15, atol=0)
        F = sp.csr_matrix((vals, fcols, frp), shape=(flat.n_emitters,) * 2)
        rs = np.asarray(F.sum(axis=1)).ravel()
        assert np.allclose(rs[np.diff(rp) > 0], 1.0, rtol=0, atol=1e-12)


def test_pinned_copy_equals_pageable_copy(hip):
    dom = H.square_domain(41)
    flat = dom.flat()
    args, _k = _args(hip, flat, 5000, seed=3)
    dd = hip.DeviceDomain(flat, 0)
    pin = hip.PinnedArrays()
    try:
        a = _trace(hip, dd, args)
        b = _trace(hip, dd, args, pinned=pin)
    finally:
        dd.close()
        pin.close()
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)


def test_lookback_stall_falls_back_to_staging(hip, monkeypatch):
    """RTHX_LB_WAIT_US=0: a row gives up its look-back wait as soon as a
    predecessor has not yet published; the call then re-traces the launch on
    the staging path.  The returned CSR must equal the staging path's (and
    the oracle's), never a misplaced direct write."""
    dom = H.square_domain(31)
    flat = dom.flat()
    args, _k = _args(hip, flat, 3000, seed=5)
    monkeypatch.setenv("RTHX_NO_LOOKBACK", "1")
    dd = hip.DeviceDomain(flat, 0)
    ref = _trace(hip, dd, args)
    monkeypatch.delenv("RTHX_NO_LOOKBACK")
    assert ref[3]["lookback_fallbacks"] == 0
    monkeypatch.setenv("RTHX_LB_WAIT_US", "0")
    fallbacks = 0
    for _ in range(3):
        got = _trace(hip, dd, args)
        fallbacks += got[3]["lookback_fallbacks"]
        for x, y in zip(ref[:3], got[:3]):
            assert np.array_equal(x, y)
        assert got[3]["nnz"] == ref[3]["nnz"] and got[3]["lost_max_row"] == ref[3]["lost_max_row"]
    assert fallbacks >= 1, "a zero wait bound never stalled"
    monkeypatch.delenv("RTHX_LB_WAIT_US")
    got = _trace(hip, dd, args)  # default bound: the direct write, no fallback
    dd.close()
    assert got[3]["lookback_fallbacks"] == 0 and got[3]["pack_ms"] < 0.05
    assert np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2])
    small = oracle.trace_exchange(flat, args, 16)
    assert np.array_equal(ref[2], small[2])


def _open_square(ndim):
    """A square whose top wall is open (rays through it are lost), so the
    look-back launch's lost-ray totals (atomics) are non-zero."""
    face = H.PolyVolume2D([(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)], [True, True, False, True], 1, 1.0, 0.0)
    face.T_in_w = [1000.0, 0.0, 0.0, 0.0]
    face.epsilon = [1.0] * 4
    face.T_in_g = -1.0
    face.q_in_g = 0.0
    return H.RayTracingDomain2D([face], [(ndim, ndim)])


def test_reused_result_across_lookback_launches(hip, monkeypatch):
    """One result object traced again and again (as bench.py does): the
    look-back words are tagged with the launch's epoch and row 0 zeroes the
    next launch's totals, so nothing is zeroed between launches.  Every call
    (growing and shrinking row counts, a staging launch in between) must
    give the counts and totals of a fresh result, and the totals must not
    accumulate over calls."""
    small, big = _open_square(23), _open_square(37)
    fs, fb = small.flat(), big.flat()
    ds, db = hip.DeviceDomain(fs, 0), hip.DeviceDomain(fb, 0)
    a_s, _k1 = _args(hip, fs, 2000, seed=11)
    a_b, _k2 = _args(hip, fb, 1500, seed=12)
    want_s, want_b = _trace(hip, ds, a_s), _trace(hip, db, a_b)
    assert want_s[3]["lost_total"] > 0 and want_b[3]["lost_total"] > 0
    res = hip.DeviceResult()
    try:
        plan = ["s", "s", "b", "s", "staging", "b", "b", "s"] + ["s"] * 8
        for step in plan:
            if step == "staging":
                monkeypatch.setenv("RTHX_NO_LOOKBACK", "1")
            dd, args, want = (db, a_b, want_b) if step == "b" else (ds, a_s, want_s)
            res.trace(dd, args)
            monkeypatch.delenv("RTHX_NO_LOOKBACK", raising=False)
            info = res.info()
            rp, cols, cnt = res.csr()
            for x, y in zip(want[:3], (rp, cols, cnt)):
                assert np.array_equal(x, y), step
            for k in ("nnz", "lost_total", "lost_max_row"):
                assert info[k] == want[3][k], (step, k)
            assert info["lookback_fallbacks"] == 0
    finally:
        res.close()
        ds.close()
        db.close()
    ref = oracle.trace_exchange(fs, a_s, 16)
    assert np.array_equal(want_s[2], ref[2]) and want_s[3]["lost_total"] == ref[3]["lost_total"]


@pytest.mark.parametrize("case", ["grey11", "transparent", "scatter"])
def test_smooth_from_device_result_equals_host_csr_smoothing(hip, case):
    """rthx_smooth_F_result (counts never leave the device) equals
    rthx_smooth_F on the host CSR of the same F_raw, to 1e-12: dense OP+AP
    (grey 11x11), the surfaces-only block (kappa = 0, n = Ns), and sparse AP."""
    from rthx.smoothing import get_w, smooth_F, smooth_F_device

    dom = {"grey11": lambda: H.square_domain(11), "transparent": lambda: H.square_domain(6, kappa=0.0),
           "scatter": lambda: H.square_domain(25, sigma_s=5.0)}[case]()
    flat = dom.flat()
    R = {"grey11": 6000, "transparent": 4000, "scatter": 150}[case]
    args, _k = _args(hip, flat, R, seed=2)
    dd = hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        rp, cols, vals = res.F()
        n = dom.num_surfaces if dom.surfaces_only else flat.n_emitters
        F = sp.csr_matrix((vals, cols, rp), shape=(flat.n_emitters,) * 2)[:n, :n].tocsr()
        w = get_w(dom)
        kw = dict(smooth_surfaces_only=dom.surfaces_only, verbose=False)
        i_host, i_dev = {}, {}
        A = smooth_F(F, w, dom.num_surfaces, info=i_host, **kw)
        h = smooth_F_device(res, n, w, dom.num_surfaces, info=i_dev, **kw)
        B = h.host()
        h.close()
    finally:
        res.close()
        dd.close()
    assert i_host["dense"] == i_dev["dense"] and i_host["k_dykstra"] == i_dev["k_dykstra"]
    assert abs(i_host["ap_iters"] - i_dev["ap_iters"]) <= 2
    assert abs(i_host["chi"] - i_dev["chi"]) <= 1e-12
    if case == "scatter":
        assert not i_dev["dense"]
    A = A.toarray() if sp.issparse(A) else A
    B = B.toarray() if sp.issparse(B) else B
    assert np.max(np.abs(A - B)) <= 1e-12


def test_mesh_keeps_F_on_device_until_read(hip):
    """mesh(): trace -> smoothing of the device counts -> GERT solve on the
    device-resident F_smooth; F_smooth crosses to the host only when read,
    and then equals the host-CSR smoothing of the returned F_raw."""
    from rthx.equilibrium import equilibrium_grey
    from rthx.smoothing import get_w, smooth_F

    dom = H.square_domain(11)
    assert dom(1_000_000, seed=11, verbose=False) is None
    assert dom._F_smooth_handle is not None and dom._F_smooth is None
    assert dom._F_raw_lazy is not None and dom._F_raw is None
    T, j, Abs, r = equilibrium_grey(dom, None)
    assert dom._F_smooth_handle is not None  # the solve read F_smooth in place
    assert abs(dom.energy_error) < 1e-4
    Fs = dom.F_smooth
    assert dom._F_smooth_handle is None and isinstance(Fs, np.ndarray)
    F_raw = dom.F_raw  # host copy on first read
    assert dom._F_raw_lazy is None and F_raw.shape == (dom.num_emitters,) * 2
    assert np.allclose(np.asarray(F_raw.sum(axis=1)).ravel(), 1.0, rtol=0, atol=1e-12)
    ref = smooth_F(F_raw, get_w(dom), dom.num_surfaces, verbose=False)
    assert np.max(np.abs(Fs - ref)) <= 1e-12
    T2, *_ = equilibrium_grey(dom, dom.F_smooth)  # the host copy is still recognised as device-resident
    np.testing.assert_allclose(T2, T, rtol=1e-12)


def _bench_line(argv, timeout=240):
    import json
    import subprocess
    import sys

    out = subprocess.run([sys.executable, H.os.path.join(H.ROOT, "bench.py")] + argv, capture_output=True, text=True,
                         timeout=timeout, cwd=H.ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("mode", ["ranks", "threads"])
def test_bench_two_gpus_as_a_plain_command(hip, mode):
    """`python bench.py --gpus 2` started as a plain process spawns its two
    ranks itself (torch.distributed.run, before any GPU call); `--mode
    threads` drives two device slots from one process.  On a one-GPU box both
    share device 0; the line is well-formed with n_gpus 2 and 2e7 rays per
    GPU slot."""
    d = _bench_line(["--gpus", "2", "--steps", "3", "--warmup", "1", "--prewarm-s", "0", "--no-cpu",
                     "--rays-per-gpu", "20000000", "--mode", mode])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["config"]["rays_per_step"] == (40_000_000 // 10605) * 10605


def test_bench_falls_back_to_blocking_steps_when_pipelined_steps_fault(hip, monkeypatch):
    """With a zero look-back wait bound (RTHX_LB_WAIT_US=0) the pipelined
    timed steps stall and are superseded unread, so bench.py times the steps
    again as blocking calls (each re-traced when needed) and says so in its
    line; two ranks decide together.  A normal run reports no faults."""
    monkeypatch.setenv("RTHX_LB_WAIT_US", "0")
    for extra in ([], ["--gpus", "2", "--rays-per-gpu", "20000000"]):
        d = _bench_line(["--steps", "4", "--warmup", "1", "--prewarm-s", "0", "--no-cpu", "--faithful-steps", "0"] + extra)
        assert d["pipelined_step_faults"] > 0 and d["step_mode"].startswith("blocking calls (fallback")
        assert d["steps_checked"] == 4 and d["value"] > 0
    monkeypatch.delenv("RTHX_LB_WAIT_US")
    d = _bench_line(["--steps", "4", "--warmup", "1", "--prewarm-s", "0", "--no-cpu", "--faithful-steps", "0"])
    assert d["pipelined_step_faults"] == 0 and d["steps_checked"] == 4
    assert d["step_mode"] == "enqueued back to back (RTHX_FLAG_ASYNC)"


@pytest.mark.parametrize("case", ["square", "greenhouse", "shard"])
def test_device_csr_equals_host_csr(hip, case):
    """rthx_result_get_device_csr / rthx_result_copy_csr_device: the block a
    collective sends from device memory (rthx.distributed.gather_result on
    NCCL groups) holds exactly the host CSR's rows -- single- and
    multi-polygon kernels, and a strided shard (rows begin + k stride)."""
    torch = pytest.importorskip("torch")
    dom = H.greenhouse_domain(n_layers=6, nx=9, ny=3, n_bins=8) if case == "greenhouse" else H.square_domain(13)
    flat = dom.flat()
    begin, stride = (1, 3) if case == "shard" else (0, 1)
    args = _args(hip, flat, 3000, seed=4, begin=begin, stride=stride)[0]
    dd = hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        rp, cols, cnt = res.csr()
        d = res.device_csr()
        assert d["device"] == 0 and d["n_parts"] == 1 and res.device == 0
        assert d["emitter_begin"] == begin and d["emitter_stride"] == stride
        assert d["nnz"] == rp[-1] and d["row_off"] and d["cols"] and d["counts"]
        row_off, pairs, _d = res.torch_csr()
        assert row_off.device.type == "cuda" and pairs.device.type == "cuda"
        rows = np.arange(begin, flat.n_emitters, stride)
        assert d["n_rows"] == rows.size
        ro = row_off.cpu().numpy()
        assert np.array_equal(np.diff(ro), np.diff(rp)[rows])
        p = pairs.cpu().numpy()
        assert np.array_equal(p[0], cols) and np.array_equal(p[1].view(np.uint32), cnt)
    finally:
        res.close()
        dd.close()


def test_direct_csr_overflow_retraces_with_exact_size(hip, monkeypatch):
    """The direct CSR is reserved from the previous launch's nnz (a guess on
    the first): rows that outgrow it write nothing, flag the overflow, and the
    host traces the launch again into buffers of the exact size.  A forced
    tiny reservation (RTHX_CSR_CAP) must give the same CSR, report one extra
    launch, and the next launch of the same result must fit."""
    dom = H.square_domain(31)
    flat = dom.flat()
    args = _args(hip, flat, 4000, seed=21)[0]
    dd = hip.DeviceDomain(flat, 0)
    try:
        want = _trace(hip, dd, args)
        assert want[3]["lookback_fallbacks"] == 0  # (worst case 1085 x 1085 entries: reserved outright)
        monkeypatch.setenv("RTHX_CSR_CAP", "1000")
        res = hip.DeviceResult()
        try:
            res.trace(dd, args)
            assert res.info()["lookback_fallbacks"] == 1
            got = res.csr()
            monkeypatch.delenv("RTHX_CSR_CAP")
            res.trace(dd, args)  # sized from the last nnz now: no second launch
            assert res.info()["lookback_fallbacks"] == 0
            again = res.csr()
        finally:
            res.close()
        for x, y, z in zip(want[:3], got, again):
            assert np.array_equal(x, y) and np.array_equal(x, z)
    finally:
        dd.close()


def test_c2_direct_csr_working_set(hip):
    """C2 (101 x 101, 1e8 rays): after the first launch the direct CSR is
    sized from the measured nnz (~30.5 M entries: ~275 MB for cols and
    counts) instead of rows x min(N, R) (800 MB)."""
    torch = pytest.importorskip("torch")
    flat = H.square_domain(101).flat()
    N = flat.n_emitters
    args = _args(hip, flat, 100_000_000 // N, seed=1, flags=hip.abi.RTHX_FLAG_DEVICE_ONLY)[0]
    dd = hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)  # first launch: guessed size (may re-trace once)
        res.trace(dd, args)
        free0 = torch.cuda.mem_get_info(0)[0]
        res2 = hip.DeviceResult()
        try:
            res2.trace(dd, args)
            res2.trace(dd, args)
            used = free0 - torch.cuda.mem_get_info(0)[0]
            nnz = res2.info()["nnz"]
        finally:
            res2.close()
        assert nnz > 2e7
        assert used < 0.5 * N * (100_000_000 // N) * 8, used  # well under the 800 MB worst case
        assert used < 400e6, used
    finally:
        res.close()
        dd.close()


def test_gather_and_broadcast_over_rccl(hip):
    """The NCCL (= RCCL on ROCm) branches of rthx.distributed on a real GPU:
    a one-rank NCCL group (a one-GPU box cannot hold two ranks on one
    device) gathers a traced result from device memory
    (rthx_result_copy_csr_device -> the tensors RCCL sends), to one rank and
    to all, and broadcasts a CSR; every form equals the host CSR."""
    torch = pytest.importorskip("torch")
    import socket

    import torch.distributed as dist
    from rthx import distributed as RD

    flat = H.square_domain(15).flat()
    N = flat.n_emitters
    args = _args(hip, flat, 2000, seed=9, begin=1, stride=2)[0]
    dd = hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        res.trace(dd, args)
        rp, cols, cnt = res.csr()
        for dst in (0, -1):
            g_rp, g_c, g_v = RD.gather_result(res, N, dst=dst)
            assert np.array_equal(g_rp, rp) and np.array_equal(g_c, cols) and np.array_equal(g_v, cnt)
        t_rp, t_c, t_v = RD.gather_result(res, N, dst=0, as_tensors=True)
        assert t_rp.device.type == "cuda" and t_c.device.type == "cuda"
        assert np.array_equal(t_v.cpu().numpy().view(np.uint32), cnt)
        h_rp, h_c, h_v = RD.gather_csr(rp, cols, cnt, N, dst=0)
        assert np.array_equal(h_rp, rp) and np.array_equal(h_c, cols) and np.array_equal(h_v, cnt)
        b_rp, b_c, b_v = RD.broadcast_csr(rp, cols, cnt, N, src=0)
        assert np.array_equal(np.asarray(b_rp), rp) and np.array_equal(np.asarray(b_c), cols)
        assert np.array_equal(np.asarray(b_v).view(np.uint32), cnt)
        # a result of several device blocks (rthx_multi_trace_exchange):
        # contiguous row blocks on the square, interleaved on the wedges;
        # every block is gathered, and torch's current device is unchanged
        for flat2, devices in ((flat, [0, 0]), (H.wedge_domain(8, 3).flat(), [0, 0, 0])):
            a2 = _args(hip, flat2, 700, seed=10, begin=1, stride=2)[0]
            md = hip.MultiDeviceDomain(flat2, devices)
            r2 = hip.DeviceResult()
            try:
                r2.trace(md, a2)
                assert r2.device_csr(0)["n_parts"] == len(devices)
                m_rp, m_c, m_v = r2.csr()
                for dst in (0, -1):
                    g_rp, g_c, g_v = RD.gather_result(r2, flat2.n_emitters, dst=dst)
                    assert np.array_equal(g_rp, m_rp) and np.array_equal(g_c, m_c) and np.array_equal(g_v, m_v)
                assert torch.cuda.current_device() == 0
            finally:
                r2.close()
                md.close()
    finally:
        dist.destroy_process_group()
        res.close()


def test_async_traces_equal_blocking_traces(hip):
    """RTHX_FLAG_ASYNC: traces enqueued back to back into one result (the
    bench's pipelined steps) read back exactly as blocking traces: the last
    one's CSR and totals, completed and checked on the first read.  A first
    trace of a shape blocks (its CSR is sized then); a pending trace that is
    traced over is superseded; a result destroyed while pending is safe; the
    device CSR hand-out and F_raw complete a pending trace too."""
    A = hip.abi
    dom = H.square_domain(21)
    flat = dom.flat()
    dd = hip.DeviceDomain(flat, 0)
    try:
        want = {}
        for seed in (5, 6):
            args, _k = _args(hip, flat, 4000, seed=seed)
            want[seed] = _trace(hip, dd, args)
        res = hip.DeviceResult()
        try:
            a5, _k5 = _args(hip, flat, 4000, seed=5, flags=A.RTHX_FLAG_ASYNC | A.RTHX_FLAG_DEVICE_ONLY)
            a6, _k6 = _args(hip, flat, 4000, seed=6, flags=A.RTHX_FLAG_ASYNC | A.RTHX_FLAG_DEVICE_ONLY)
            res.trace(dd, a5)  # (first trace of the shape: blocks)
            for _ in range(4):
                res.trace(dd, a5)
            res.trace(dd, a6)  # superseded by the next one
            res.trace(dd, a5)
            info = res.info()
            rp, cols, cnt = res.csr()
            w = want[5]
            assert np.array_equal(rp, w[0]) and np.array_equal(cols, w[1]) and np.array_equal(cnt, w[2])
            for k in ("nnz", "lost_total", "lost_max_row", "rays_traced", "rows_traced"):
                assert info[k] == w[3][k], k
            assert info["lookback_fallbacks"] == 0 and info["trace_ms"] > 0
            # four async a5 and the a6 were replaced unread; none faulted
            assert info["superseded"] == 5 and info["superseded_faults"] == 0
            # the device CSR of a pending trace
            res.trace(dd, a6)
            d = res.device_csr()
            assert d["nnz"] == want[6][3]["nnz"]
            rp6, c6, n6 = res.csr()
            assert np.array_equal(c6, want[6][1]) and np.array_equal(n6, want[6][2])
            # F_raw of a pending trace
            res.trace(dd, a5)
            frp, fc, fv = res.F()
            assert np.array_equal(fc, w[1]) and np.all(fv > 0)
            res.trace(dd, a6)  # left pending: closing must be safe
        finally:
            res.close()
    finally:
        dd.close()


def test_superseded_async_faults_are_counted(hip, monkeypatch):
    """async steps that a later step replaces unread are
    checked too.  With a zero look-back wait bound (RTHX_LB_WAIT_US=0) a step
    stalls as soon as a row has to wait; its stall flag is carried by the
    next launch's row 0 into that launch's totals (TallyParams::check_prev)
    and reported as superseded_faults, while the last step -- traced with the
    default bound -- still equals the blocking trace.  A replaced step that
    the next trace cannot chain (a staged launch, which frees the look-back
    totals) is read back on the host first.  Each replaced step is counted
    exactly once."""
    A = hip.abi
    dom = H.square_domain(31)
    flat = dom.flat()
    dd = hip.DeviceDomain(flat, 0)
    try:
        b, _kb = _args(hip, flat, 3000, seed=5)
        ref = _trace(hip, dd, b)
        a, _ka = _args(hip, flat, 3000, seed=5, flags=A.RTHX_FLAG_ASYNC | A.RTHX_FLAG_DEVICE_ONLY)
        res = hip.DeviceResult()
        try:
            res.trace(dd, b)  # (sizes the shape: later async calls enqueue)
            k = 8
            faults = 0
            for form in ("chained", "absorbed"):
                monkeypatch.setenv("RTHX_LB_WAIT_US", "0")
                for _ in range(k):
                    res.trace(dd, a)
                monkeypatch.delenv("RTHX_LB_WAIT_US")
                if form == "chained":
                    res.trace(dd, a)  # same shape: row 0 folds in the replaced step's flags
                    info = res.info()
                    rp, cols, cnt = res.csr()
                    assert np.array_equal(rp, ref[0]) and np.array_equal(cols, ref[1]) and np.array_equal(cnt, ref[2])
                else:
                    other, _ko = _args(hip, flat, 2000, seed=5)
                    monkeypatch.setenv("RTHX_NO_LOOKBACK", "1")
                    res.trace(dd, other)  # the staging path: the replaced step is read back on the host first
                    monkeypatch.delenv("RTHX_NO_LOOKBACK")
                    info = res.info()
                    res.trace(dd, b)
                    assert res.info()["superseded"] == 0
                assert info["superseded"] == k, (form, info["superseded"])
                assert 0 <= info["superseded_faults"] <= k
                faults += info["superseded_faults"]
            assert faults >= 1, "a zero wait bound never stalled a replaced step"
        finally:
            res.close()
    finally:
        dd.close()


@pytest.mark.parametrize("shape", ["full", "shard", "multi"])
def test_F_csc_equals_host_transpose(hip, shape):
    """rthx_result_copy_F_csc (F_raw as Julia's SparseMatrixCSC layout,
    transposed on the device by a radix sort of (column, row) keys; several
    devices' results on the host) equals the host transpose of
    rthx_result_copy_F's CSR exactly, indices counted from 0 and from 1."""
    import scipy.sparse as sp

    flat = H.square_domain(21, kappa=0.7).flat()
    N = flat.n_emitters
    begin, stride = (1, 3) if shape == "shard" else (0, 1)
    args, _k = hip.make_args(0, 3001, H.NUDGE, 4, begin, N, stride)
    dd = hip.MultiDeviceDomain(flat, [0, 0]) if shape == "multi" else hip.DeviceDomain(flat, 0)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        rp, cols, vals = res.F()
        ref = sp.csr_matrix((vals, cols, rp), shape=(N, N)).tocsc()
        ref.sort_indices()
        for base in (0, 1):
            cp, rv, nz = res.F_csc(base)
            assert np.array_equal(cp - base, ref.indptr)
            assert np.array_equal(rv - base, ref.indices)
            assert np.array_equal(nz, ref.data)
    finally:
        res.close()
        dd.close()
