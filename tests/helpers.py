"""Test helpers: reference test geometries and a numpy restatement of the grey
GERT solve used to pin the tracer against the reference's own known answers.

Test infrastructure only (the solver is the reference's host code, which stays
on the host and out of this package's scope: SURVEY.md §2 row 8).
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytraceheattransfer.jl_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

from rthx import PolyVolume2D, RayTracingDomain2D  # noqa: E402

STEFAN_BOLTZMANN = 5.670374419e-8  # src/RayTraceHeatTransfer.jl:20
NUDGE = 10_000 * np.finfo(np.float64).eps  # multiDispatchRayTrace2D.jl:10
GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def square_face(kappa=1.0, sigma_s=0.0, rotation=0.0, T_walls=(1000.0, 0.0, 0.0, 0.0), epsilon=1.0,
                n_bins=1):
    """createSquareDomain2D's face (test/test_2d_grey.jl:41-92)."""
    base = [(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)]
    if rotation != 0.0:
        c, s = math.cos(rotation), math.sin(rotation)
        verts = [((x - 0.5) * c - (y - 0.5) * s + 0.5, (x - 0.5) * s + (y - 0.5) * c + 0.5) for x, y in base]
    else:
        verts = base
    face = PolyVolume2D(verts, [True] * 4, n_bins, kappa, sigma_s)
    face.T_in_w = list(T_walls)
    face.epsilon = [epsilon] * 4
    face.T_in_g = -1.0
    face.q_in_g = 0.0
    return face


def square_domain(ndim=11, **kw) -> RayTracingDomain2D:
    return RayTracingDomain2D([square_face(**kw)], [(ndim, ndim)])


def wedge_domain(n_wedges=16, ndim=2, kappa=1.0, T_half=(1000.0, 0.0), sigma_s=0.0, epsilon=1.0):
    """Circle of triangle wedges around the origin (test/test_triangle_mesh.jl:1-46).

    Outer walls solid, spokes open; the first half of the wedges' outer walls
    at T_half[0], the rest at T_half[1].
    """
    faces = []
    for k in range(n_wedges):
        a0 = 2 * math.pi * k / n_wedges
        a1 = 2 * math.pi * (k + 1) / n_wedges
        verts = [(0.0, 0.0), (math.cos(a0), math.sin(a0)), (math.cos(a1), math.sin(a1))]
        f = PolyVolume2D(verts, [False, True, False], 1, kappa, sigma_s)
        T = T_half[0] if k < n_wedges // 2 else T_half[1]
        f.T_in_w = [0.0, T, 0.0]
        f.epsilon = [epsilon] * 3
        f.T_in_g = -1.0
        f.q_in_g = 0.0
        faces.append(f)
    return RayTracingDomain2D(faces, [(ndim, ndim)] * n_wedges)


def element_arrays(dom):
    """Per-element (global order) properties as populateWorkspace! gathers them
    (src/HeatTransfer/equilibrium/WorkspaceStructs.jl:68-118), bin 1."""
    ns, nv = dom.num_surfaces, dom.num_volumes
    area = np.zeros(ns); eps = np.zeros(ns); Tw = np.zeros(ns); qw = np.zeros(ns)
    vol = np.zeros(nv); kap = np.zeros(nv); omg = np.zeros(nv); Tg = np.zeros(nv); qg = np.zeros(nv)
    for (c, f, w), s in dom.surface_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        e = face.epsilon[w - 1]
        area[s - 1] = face.area[w - 1]
        eps[s - 1] = float(np.atleast_1d(e)[0])
        Tw[s - 1] = face.T_in_w[w - 1]
        qw[s - 1] = face.q_in_w[w - 1]
    for (c, f), v in dom.volume_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        k = float(np.atleast_1d(face.kappa_g)[0]); s_ = float(np.atleast_1d(face.sigma_s_g)[0])
        vol[v - 1] = face.volume
        kap[v - 1] = k
        omg[v - 1] = s_ / (k + s_) if k + s_ > 0 else 0.0
        Tg[v - 1] = face.T_in_g
        qg[v - 1] = face.q_in_g
    return dict(area=area, eps=eps, Tw=Tw, qw=qw, vol=vol, kappa=kap, omega=omg, Tg=Tg, qg=qg)


def solve_grey(dom, F):
    """equilibriumGrey2D!, src/HeatTransfer/equilibrium/equilibriumGrey2D.jl:80-211
    (dense/sparse direct solve of (I - diag(coeff) F^T) j = h).  Returns
    (T_surfaces, T_volumes, energy_error)."""
    a = element_arrays(dom)
    ns = dom.num_surfaces
    nv = 0 if dom.surfaces_only else dom.num_volumes
    n = ns + nv
    F = sp.csr_matrix(F)[:n, :n]
    q_known = np.concatenate([(a["Tw"] < 0).astype(int), (a["Tg"][:nv] < 0).astype(int)])
    E = np.zeros(n); Q = np.zeros(n)
    for i in range(ns):
        if q_known[i] == 0:
            E[i] = a["eps"][i] * STEFAN_BOLTZMANN * a["area"][i] * a["Tw"][i] ** 4
        else:
            Q[i] = a["qw"][i]
    for v in range(nv):
        i = ns + v
        if q_known[i] == 0:
            E[i] = 4 * a["kappa"][v] * STEFAN_BOLTZMANN * a["vol"][v] * a["Tg"][v] ** 4
        else:
            Q[i] = a["qg"][v]
    b = np.zeros(n)
    if np.any(a["omega"][:nv] > 1e-6) or np.sum(a["eps"]) < n:
        b[:ns] = 1.0 - a["eps"]
        b[ns:] = a["omega"][:nv]
    h = np.where(q_known == 1, Q, E)
    coeff = np.where(q_known == 1, 1.0, b)
    M = sp.identity(n, format="csr") - sp.diags(coeff) @ F.T.tocsr()
    j = spla.spsolve(M.tocsc(), h)
    g = F.T @ j
    r = b * g
    absorbed = (1.0 - b) * g
    T = np.zeros(n)
    for i in range(ns):
        e = max(j[i] - r[i], 0.0)
        T[i] = (e / (a["eps"][i] * STEFAN_BOLTZMANN * a["area"][i])) ** 0.25 if a["eps"][i] > 0 else 0.0
    for v in range(nv):
        i = ns + v
        e = max(j[i] - r[i], 0.0)
        if a["kappa"][v] > 0 and a["vol"][v] > 0:
            T[i] = (e / (4 * a["kappa"][v] * a["vol"][v] * STEFAN_BOLTZMANN)) ** 0.25
    energy_error = float(np.sum(j - r - absorbed))
    return T[:ns], T[ns:], energy_error


def centerline_source_function(dom, ndim, T_hot=1000.0):
    """extractCenterlineTemperatures + dimensionlessSourceFunction (test/test_2d_grey.jl:94-118)."""
    _, Tg, _ = solve_grey(dom, dom.F_raw)
    grid = Tg.reshape(ndim, ndim)  # row m (y) major, n (x) fastest
    col = (ndim + 1) // 2 - 1
    return (grid[:, col] / T_hot) ** 4


def line_interpolation(xd, yd, x):
    """lineInterpolation (test/test_2d_grey.jl:124-162), constant extrapolation."""
    return np.interp(x, xd, yd)


def reciprocity_weights(dom, bin0=0):
    """w = [wall length; 4 beta V] (smoothExchangeFactors.jl:320-341, get_w)."""
    flat = dom.flat()
    ns = dom.num_surfaces
    w = np.zeros(dom.num_emitters)
    w[:ns] = dom.surface_areas
    beta = flat.beta.reshape(flat.n_bins, flat.n_fine)[bin0]
    w[ns:] = 4.0 * beta * flat.fine_volume
    return w


# --------------------------------------------------------------------------
# statistical / analytic checks
# --------------------------------------------------------------------------
def csr_rows_subset(row_ptr, cols, counts, n, rows):
    """The CSR (row_ptr[n+1], cols, counts) restricted to `rows` (ascending):
    every other row empty, as a strided shard of the same trace returns it."""
    rows = np.asarray(rows, dtype=np.int64)
    lens = np.zeros(n, dtype=np.int64)
    lens[rows] = row_ptr[rows + 1] - row_ptr[rows]
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=rp[1:])
    idx = np.concatenate([np.arange(row_ptr[r], row_ptr[r + 1]) for r in rows]) if len(rows) else np.zeros(0, np.int64)
    return rp, cols[idx], counts[idx]


def counts_matrix(row_ptr, cols, counts, n):
    return sp.csr_matrix((counts.astype(np.float64), cols.astype(np.int64), row_ptr.astype(np.int64)), shape=(n, n))


def surface_segments(dom):
    """[(a, b)] end points of every surface element, CCW along its polygon."""
    segs = [None] * dom.num_surfaces
    for (c, f, w), s in dom.surface_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        a = face.vertices[w - 1]
        b = face.vertices[w % face.n]
        segs[s - 1] = (np.array(a), np.array(b))
    return segs


def crossed_strings(seg1, seg2):
    """View factor between two CCW boundary segments of a convex enclosure
    (Hottel crossed strings); 0 for collinear segments."""
    a1, b1 = seg1
    a2, b2 = seg2
    d1 = b1 - a1
    cross = lambda u, v: u[0] * v[1] - u[1] * v[0]
    if abs(cross(d1, a2 - a1)) < 1e-12 and abs(cross(d1, b2 - a1)) < 1e-12:
        return 0.0
    L = np.linalg.norm
    crossed = L(a1 - a2) + L(b1 - b2)
    uncrossed = L(a1 - b2) + L(b1 - a2)
    return (crossed - uncrossed) / (2 * L(d1))


def reciprocity_z(C, R, w, min_count=50):
    """z-scores of w_i F_ij - w_j F_ji for pairs where both counts >= min_count
    (F = C/R, binomial variances).  Reciprocity holds only if emission uses the
    un-normalised in-plane directions of the reference."""
    C = sp.csr_matrix(C, dtype=np.float64)
    C.data[C.data < min_count] = 0
    C.eliminate_zeros()
    Ct = C.T.tocsr()
    A = C.multiply(Ct.astype(bool)).tocsr()
    B = Ct.multiply(C.astype(bool)).tocsr()
    A.sort_indices()
    B.sort_indices()
    assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
    i = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    j = A.indices
    m = i < j
    i, j, c, cji = i[m], j[m], A.data[m], B.data[m]
    Fij, Fji = c / R, cji / R
    a, b = w[i] * Fij, w[j] * Fji
    var = w[i] ** 2 * Fij * (1 - Fij) / R + w[j] ** 2 * Fji * (1 - Fji) / R
    return (a - b) / np.sqrt(var)


def element_keys(dom, nd=9):
    """Geometric key per global element (wall midpoint / cell midpoint), for
    matching elements of two meshings of the same region."""
    keys = [None] * dom.num_emitters
    for (c, f, w), s in dom.surface_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        m = face.wallMidPoints[w - 1]
        keys[s - 1] = ("s", round(m[0], nd), round(m[1], nd))
    ns = dom.num_surfaces
    for (c, f), v in dom.volume_mapping.items():
        m = dom.fine_mesh[c - 1][f - 1].midPoint
        keys[ns + v - 1] = ("v", round(m[0], nd), round(m[1], nd))
    return keys


def greenhouse_domain(n_layers=67, nx=201, ny=3, n_bins=8, scale_height=15_900.0 / 100_000.0,
                      kappa_vis=0.01, kappa_ir=100.0, uniform=False):
    """BASELINE configs[4] geometry: a 1x1 stack of coarse
    layers, side walls solid, bottom of layer 1 and top of the last layer
    solid, interfaces open; per-band kappa(y) = rho(y_mid) (k_ir s_b + k_vis
    (1 - s_b)), s_b = 1/(1 + (4 um / lambda_b)^6) (readme.md:227-247),
    log-spaced bands between 1 nm and 1 m (readme.md:202-204)."""
    edges = 10 ** np.linspace(-9, 0, n_bins + 1)
    centers = np.sqrt(edges[:-1] * edges[1:])
    sig = 1 / (1 + (4e-6 / centers) ** 6)
    faces = []
    for j in range(n_layers):
        y0, y1 = j / n_layers, (j + 1) / n_layers
        rho = math.exp(-((y0 + y1) / 2) / scale_height)
        kap = rho * (kappa_ir * sig + kappa_vis * (1 - sig))
        if uniform:  # (every layer the same kappa: traceRayUniform)
            kap = np.full(n_bins, 0.7)
        f = PolyVolume2D([(0.0, y0), (1.0, y0), (1.0, y1), (0.0, y1)], [j == 0, True, j == n_layers - 1, True],
                         n_bins, kap, np.zeros(n_bins))
        f.epsilon = [np.ones(n_bins) for _ in range(4)]
        f.T_in_g = -1.0
        faces.append(f)
    return RayTracingDomain2D(faces, [(nx, ny)] * n_layers)


def layered_slab_domain(kappas, W=100.0, nx=21):
    """A W x 1 slab between two black plates cut into len(kappas) horizontal
    layers of equal height, layer j with extinction kappas[j] (a coarse
    rectangle each, meshed nx x 2; side walls solid, interfaces open): the
    traceRayVariable walk (traceRay.jl:73-147) across every layer.  Plate
    to plate, a cold non-scattering slab transmits 2 E3(tau) of a Lambert
    emitter's rays, tau = sum(kappas) / len(kappas) (slab_transmission)."""
    L = len(kappas)
    faces = []
    for j, k in enumerate(kappas):
        y0, y1 = j / L, (j + 1) / L
        f = PolyVolume2D([(0.0, y0), (W, y0), (W, y1), (0.0, y1)], [j == 0, True, j == L - 1, True], 1, float(k), 0.0)
        f.epsilon = [1.0] * 4
        f.T_in_g = -1.0
        faces.append(f)
    return RayTracingDomain2D(faces, [(nx, 2)] * L)


def slab_transmission(dom, row_ptr, cols, counts, n_central=5):
    """(mean, standard error) over the n_central middle bottom-plate elements
    of the fraction of each row's tallied rays absorbed by the top plate."""
    L, nx = len(dom.fine_mesh), len(dom.fine_mesh[0]) // 2  # (fine faces x fastest: row 1 then row 2)
    top = np.array(sorted(dom.surface_mapping[(L, f, 3)] - 1 for f in range(nx + 1, 2 * nx + 1)))
    lo = (nx - n_central) // 2 + 1
    fr = []
    for f in range(lo, lo + n_central):
        g = dom.surface_mapping[(1, f, 1)] - 1
        c = cols[row_ptr[g]:row_ptr[g + 1]]
        n = counts[row_ptr[g]:row_ptr[g + 1]].astype(np.float64)
        fr.append(n[np.isin(c, top)].sum() / n.sum())
    fr = np.array(fr)
    return float(fr.mean()), float(fr.std(ddof=1) / math.sqrt(len(fr)))


def quad_lattice_domain(ncx=2, ncy=3, nxf=4, nyf=3, kappa=0.8):
    """A unit square cut into an ncx x ncy lattice of coarse squares (outer
    walls solid, interior walls open), each meshed nxf x nyf: a multi-polygon
    lattice with more than one coarse column (MLAT kernels)."""
    faces = []
    for j in range(ncy):
        for i in range(ncx):
            x0, x1, y0, y1 = i / ncx, (i + 1) / ncx, j / ncy, (j + 1) / ncy
            f = PolyVolume2D([(x0, y0), (x1, y0), (x1, y1), (x0, y1)],
                             [j == 0, i == ncx - 1, j == ncy - 1, i == 0], 1, kappa * (1 + 0.3 * ((i + j) % 2)), 0.0)
            f.T_in_g = -1.0
            faces.append(f)
    return RayTracingDomain2D(faces, [(nxf, nyf)] * len(faces))


def icosphere(level=2, radius=0.3, center=(0.5, 0.5, 0.5)):
    """Triangles of a subdivided icosahedron projected on a sphere:
    20 * 4**level faces, counter-clockwise seen from outside."""
    t = (1 + 5 ** 0.5) / 2
    V = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    V = [np.array(v, dtype=float) / np.linalg.norm(v) for v in V]
    F = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    for _ in range(level):
        cache = {}

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = V[a] + V[b]
                V.append(m / np.linalg.norm(m))
                cache[key] = len(V) - 1
            return cache[key]

        F = [f for a, b, c in F for f in ((a, mid(a, b), mid(c, a)), (b, mid(b, c), mid(a, b)),
                                          (c, mid(c, a), mid(b, c)), (mid(a, b), mid(b, c), mid(c, a)))]
    c = np.asarray(center, dtype=float)
    return np.array([[c + radius * V[i] for i in f] for f in F])


def cube_icosphere_scene(ndim=10, level=3, radius=0.3):
    """BASELINE configs[3]: the unit cube (faces split ndim x ndim, rays leave
    inward) around a centred icosphere (rays leave outward).  Returns
    (xyz[n][4][3], nv[n], normals[n][3], n_cube)."""
    from rthx.domain3d import mesh_faces

    ref = json.load(open(os.path.join(GOLDEN, "reference_3d.json")))
    pts = np.array(ref["cube_points"])
    faces = np.array(ref["cube_faces"]) - 1
    polys, normals = [], []
    centre = np.array([0.5, 0.5, 0.5])
    for (p1, p2, p3, p4) in mesh_faces(pts, faces, ndim):
        for k in range(len(p1)):
            q = np.array([p1[k], p2[k], p3[k], p4[k]])
            polys.append(q)
            normals.append(centre - q.mean(axis=0))
    n_cube = len(polys)
    for tri in icosphere(level, radius):
        q = np.zeros((4, 3))
        q[:3] = tri
        q[3] = tri[2]
        polys.append(q)
        normals.append(tri.mean(axis=0) - centre)
    nv = np.array([4] * n_cube + [3] * (len(polys) - n_cube), dtype=np.int32)
    return np.array(polys), nv, np.array(normals), n_cube


def cube_icosphere_groups(ndim=10, level=3):
    """Coplanar groups of cube_icosphere_scene: the ndim x ndim sub-faces of
    each cube face form one group (face-major, contiguous); every sphere
    triangle is its own group."""
    n_cube = 6 * ndim * ndim
    n_sph = 20 * 4 ** level
    return np.concatenate([np.arange(n_cube) // (ndim * ndim), 6 + np.arange(n_sph)]).astype(np.int32)



# --------------------------------------------------------------------------
# the reference's remaining known answers (tests/golden/reference_known_answers.json)
# --------------------------------------------------------------------------
def known_answers():
    return golden("reference_known_answers.json")


def rect_domain(W, H, nx, ny, kappa, T_in_w, epsilon, q_in_w=(0.0, 0.0, 0.0, 0.0), sigma_s=0.0):
    """One W x H rectangle meshed nx x ny, all walls solid (walls: 1 bottom,
    2 right, 3 top, 4 left), as the reference's diffusion and reflecting-wall
    tests build it (test/test_2d_diffusion.jl:29-40,
    test/test_2d_grey_reflecting.jl:51-68,:102-113)."""
    face = PolyVolume2D([(0.0, 0.0), (W, 0.0), (W, H), (0.0, H)], [True] * 4, 1, kappa, sigma_s)
    face.T_in_w = [float(t) for t in T_in_w]
    face.q_in_w = [float(q) for q in q_in_w]
    face.epsilon = [float(e) for e in epsilon]
    face.T_in_g = -1.0
    face.q_in_g = 0.0
    return RayTracingDomain2D([face], [(nx, ny)])


def diffusion_domain():
    d = known_answers()["diffusion"]
    n = d["N_side"]
    return rect_domain(d["aspect"], 1.0, n, n, d["beta"], [d["T_hot"], 0.0, 0.0, 0.0], [1.0] * 4)


def diffusion_S(z, beta, D, eps1, eps2, E1, E2):
    """diffusion_S (test/test_2d_diffusion.jl:19-23)."""
    q = (E1 - E2) / (3 * beta * D / 4 + 1 / eps1 + 1 / eps2 - 1)
    Eb1 = E1 + q * (0.5 - 1 / eps1)
    return Eb1 - (3 * beta * z / 4) * q


def diffusion_centerline_rms(dom, T_gas):
    """centerline_rms_S (test/test_2d_diffusion.jl:43-49): the column of cells
    at x index (N-1) div 2 + 1 (fine faces x fastest), S = (T/T_hot)^4
    against diffusion_S at the cell-centre taus."""
    d = known_answers()["diffusion"]
    n = d["N_side"]
    grid = np.asarray(T_gas).reshape(n, n)  # [y][x]
    Tc = grid[:, (n - 1) // 2]
    S = (Tc / d["T_hot"]) ** 4
    taus = np.linspace(1 / (2 * n), 1 - 1 / (2 * n), n)
    Sref = diffusion_S(taus, d["beta"], 1.0, 1.0, 1.0, 1.0, 0.0)
    return float(np.sqrt(np.mean((S - Sref) ** 2)))


def reflecting_domain():
    d = known_answers()["reflecting_energy"]
    return rect_domain(1.0, 1.0, d["Ndim"], d["Ndim"], d["kappa"], d["T_in_w"], d["epsilon"])


def plates_domain():
    d = known_answers()["parallel_plates"]
    return rect_domain(d["W"], d["H"], d["Nx"], d["Ny"], d["kappa"], [d["T_hot"], d["T_cold"], d["T_cold"], d["T_cold"]],
                       [d["eps"], 1.0, d["eps"], 1.0])


def plates_flux(dom, q_surf):
    """(mean q_w / area over the central bottom-wall elements, textbook q)
    (test/test_2d_grey_reflecting.jl:115-136): fine faces 1..Nx are the
    bottom row, wall 1 their hot wall."""
    d = known_answers()["parallel_plates"]
    nx = d["Nx"]
    q_text = STEFAN_BOLTZMANN * (d["T_hot"] ** 4 - d["T_cold"] ** 4) / (2 / d["eps"] - 1)
    n_central = max(1, nx // 5)
    lo = (nx - n_central) // 2 + 1
    vals = []
    for col in range(lo, lo + n_central):
        s = dom.surface_mapping[(1, col, 1)] - 1
        face = dom.fine_mesh[0][col - 1]
        vals.append(q_surf[s] / face.area[0])
    return float(np.mean(vals)), q_text


def solve_grey_full(dom, F):
    """solve_grey plus the per-element powers writeResultsToDomainGrey! stores
    (equilibriumGrey2D.jl:176-211): returns (T, q, energy_error) in global
    element order, q = e - Abs (net emitted power)."""
    a = element_arrays(dom)
    ns, nv = dom.num_surfaces, dom.num_volumes
    n = ns + nv
    F = sp.csr_matrix(F)[:n, :n]
    q_known = np.concatenate([(a["Tw"] < 0).astype(int), (a["Tg"] < 0).astype(int)])
    E = np.zeros(n); Q = np.zeros(n)
    E[:ns] = np.where(q_known[:ns] == 0, a["eps"] * STEFAN_BOLTZMANN * a["area"] * np.maximum(a["Tw"], 0) ** 4, 0)
    Q[:ns] = np.where(q_known[:ns] == 1, a["qw"], 0)
    E[ns:] = np.where(q_known[ns:] == 0, 4 * a["kappa"] * STEFAN_BOLTZMANN * a["vol"] * np.maximum(a["Tg"], 0) ** 4, 0)
    Q[ns:] = np.where(q_known[ns:] == 1, a["qg"], 0)
    b = np.zeros(n)
    if np.any(a["omega"] > 1e-6) or np.sum(a["eps"]) < n:
        b[:ns] = 1.0 - a["eps"]
        b[ns:] = a["omega"]
    h = np.where(q_known == 1, Q, E)
    coeff = np.where(q_known == 1, 1.0, b)
    M = sp.identity(n, format="csr") - sp.diags(coeff) @ F.T.tocsr()
    j = spla.spsolve(M.tocsc(), h)
    g = F.T @ j
    r = b * g
    Abs = (1.0 - b) * g
    e = np.maximum(j - r, 0.0)
    T = np.zeros(n)
    T[:ns] = np.where(a["eps"] > 0, (e[:ns] / (np.maximum(a["eps"], 1e-300) * STEFAN_BOLTZMANN * a["area"])) ** 0.25, 0)
    kv = a["kappa"] * a["vol"]
    T[ns:] = np.where(kv > 0, (e[ns:] / (4 * np.maximum(kv, 1e-300) * STEFAN_BOLTZMANN)) ** 0.25, 0)
    return T, e - Abs, float(np.sum(j - r - Abs))


def icosphere_mesh(level):
    """icosphere_mesh (readme.md:532-589): the readme's icosahedron (vertices
    normalised, its 20 faces in its order) subdivided `level` times, midpoints
    shared through a cache keyed on the sorted vertex pair and appended in
    first-use order; each face -> (a, ab, ca), (ab, b, bc), (ca, bc, c),
    (ab, bc, ca).  Returns (points[n][3], faces[m][3] 1-based)."""
    ico = known_answers()["icosphere"]
    pts = [np.asarray(p, dtype=float) / np.linalg.norm(p) for p in ico["ico_points_raw"]]
    faces = [tuple(f) for f in ico["faces"]]
    for _ in range(level):
        cache = {}
        new = list(pts)

        def mid(i, j):
            key = (min(i, j), max(i, j))
            if key in cache:
                return cache[key]
            m = (pts[i - 1] + pts[j - 1]) / 2
            new.append(m / np.linalg.norm(m))
            cache[key] = len(new)
            return len(new)

        nf = []
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (ab, b, bc), (ca, bc, c), (ab, bc, ca)]
        pts, faces = new, nf
    return np.array(pts), np.array(faces, dtype=np.int64)


def icosphere_caps(points, faces, n_cap):
    """The readme's hot / cold caps and equator (readme.md:663-697): the n_cap
    triangles with the highest / lowest centroid z (partialsortperm: stable,
    ties by index), and the equilibrium triangle with the smallest |z|
    (argmin: first)."""
    zc = np.array([points[f - 1].mean(axis=0)[2] for f in faces])
    order = np.argsort(-zc, kind="stable")
    hot = order[:n_cap]
    cold = np.argsort(zc, kind="stable")[:n_cap]
    eq_ids = np.setdiff1d(np.arange(len(faces)), np.concatenate([hot, cold]))
    equator = int(eq_ids[np.argmin(np.abs(zc[eq_ids]))])
    return hot, cold, equator


def vf3d_clamp_affected(xyz, nv):
    """Pairs whose analytic view factor (viewFactor3D.jl:133-190, restated by
    oracle_view_factors_3d and rthx_view_factors_3d) passes through the
    reference's cos(alpha) clamp: some edge pair counts as skew
    (edgePairParameters3D.jl: 1 - cos^2 > 10 eps) with |cos alpha| > 0.999,
    which viewFactor3D.jl:157 clamps to 0.999 -- alpha 2.56 deg instead of
    the true, smaller angle.  Nearly parallel edges of nearby triangles of a
    refined sphere fall there, and their terms come out far off (icosphere
    level 3: a row of F sums to 10).  Returns an n x n bool mask."""
    n = len(nv)
    E = np.zeros((n, 4, 3))
    valid = np.zeros((n, 4), dtype=bool)
    for k in range(n):
        m = int(nv[k])
        P = xyz[k, :m]
        e = np.roll(P, -1, axis=0) - P
        E[k, :m] = e / np.linalg.norm(e, axis=1)[:, None]
        valid[k, :m] = True
    c = np.einsum("aik,bjk->abij", E, E)
    skew = (1.0 - c * c) > 10 * np.finfo(np.float64).eps
    hit = skew & (np.abs(c) > 0.999) & valid[:, None, :, None] & valid[None, :, None, :]
    aff = np.any(hit, axis=(2, 3))
    np.fill_diagonal(aff, False)
    return aff


_DUNAVANT5 = (np.array([[1 / 3, 1 / 3, 1 / 3],
                        [0.059715871789770, 0.470142064105115, 0.470142064105115],
                        [0.470142064105115, 0.059715871789770, 0.470142064105115],
                        [0.470142064105115, 0.470142064105115, 0.059715871789770],
                        [0.797426985353087, 0.101286507323456, 0.101286507323456],
                        [0.101286507323456, 0.797426985353087, 0.101286507323456],
                        [0.101286507323456, 0.101286507323456, 0.797426985353087]]),
              np.array([0.225, 0.132394152788506, 0.132394152788506, 0.132394152788506,
                        0.125939180544827, 0.125939180544827, 0.125939180544827]))


def _triangle_quadrature(tri, levels=3):
    """Points and weights (summing to the area) of the degree-5 Dunavant rule
    on the 4**levels midpoint sub-triangles of `tri`."""
    tris = [np.asarray(tri, dtype=np.float64)]
    for _ in range(levels):
        nxt = []
        for a, b, c in tris:
            ab, bc, ca = (a + b) / 2, (b + c) / 2, (c + a) / 2
            nxt += [np.array([a, ab, ca]), np.array([ab, b, bc]), np.array([ca, bc, c]), np.array([ab, bc, ca])]
        tris = nxt
    T = np.array(tris)
    bary, w = _DUNAVANT5
    pts = np.einsum("pk,tkd->tpd", bary, T).reshape(-1, 3)
    area = 0.5 * np.linalg.norm(np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]), axis=1)
    return pts, (area[:, None] * w[None, :]).ravel()


def view_factor_quadrature(tri_a, n_a, tri_b, n_b, levels=3):
    """F_ab = (1 / A_a) int_a int_b cos(theta_a) cos(theta_b) / (pi r^2) by
    product quadrature (independent of the contour-integral formula; for
    triangles that share no vertex).  n_a, n_b: the sides the faces see."""
    pa, wa = _triangle_quadrature(tri_a, levels)
    pb, wb = _triangle_quadrature(tri_b, levels)
    na = np.asarray(n_a, dtype=np.float64) / np.linalg.norm(n_a)
    nb = np.asarray(n_b, dtype=np.float64) / np.linalg.norm(n_b)
    d = pb[None, :, :] - pa[:, None, :]
    r2 = np.einsum("abk,abk->ab", d, d)
    ca = np.einsum("abk,k->ab", d, na)
    cb = -np.einsum("abk,k->ab", d, nb)
    k = np.where((ca > 0) & (cb > 0), ca * cb / (np.pi * r2 * r2), 0.0)
    return float(wa @ k @ wb / wa.sum())


def box_scene(lines, level=None, radius=0.25, center=None, perturb=0.0, seed=0, spheres=None):
    """A closed box whose six faces are lattices of quads over the given
    lattice lines (lines[k]: sorted coordinates along axis k, first and last
    = the box), every face one coplanar group (rays leave inward), optionally
    an icosphere of `level` inside (each triangle its own group, rays leave
    outward).  `perturb` moves the interior lattice lines by up to that
    fraction of a cell (a non-uniform lattice); `spheres`: more icospheres,
    (level, radius, centre) each.  Returns (xyz, nv, normals, groups,
    n_hull_polygons)."""
    rng = np.random.default_rng(seed)
    L = [np.array(l, dtype=np.float64) for l in lines]
    if perturb:
        for k in range(3):
            d = np.diff(L[k])
            L[k][1:-1] += perturb * rng.uniform(-0.5, 0.5, len(L[k]) - 2) * np.minimum(d[:-1], d[1:])
    lo = np.array([l[0] for l in L])
    hi = np.array([l[-1] for l in L])
    c = (lo + hi) / 2 if center is None else np.asarray(center, dtype=np.float64)
    polys, normals, groups = [], [], []
    gid = 0
    for k in range(3):
        u, v = (k + 1) % 3, (k + 2) % 3
        for side in (0, 1):
            plane = hi[k] if side else lo[k]
            for j in range(len(L[v]) - 1):
                for i in range(len(L[u]) - 1):
                    q = np.zeros((4, 3))
                    for m, (a, b) in enumerate([(i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)]):
                        q[m, k] = plane
                        q[m, u] = L[u][a]
                        q[m, v] = L[v][b]
                    polys.append(q)
                    nrm = np.zeros(3)
                    nrm[k] = -1.0 if side else 1.0
                    normals.append(nrm)
                    groups.append(gid)
            gid += 1
    n_hull = len(polys)
    objs = list(spheres or []) + ([(level, radius, c)] if level is not None else [])
    for lvl, rad, cen in objs:
        cen = np.asarray(cen, dtype=np.float64)
        for tri in icosphere(lvl, rad, cen):
            q = np.zeros((4, 3))
            q[:3] = tri
            q[3] = tri[2]
            polys.append(q)
            normals.append(tri.mean(axis=0) - cen)
            groups.append(gid)
            gid += 1
    nv = np.array([4] * n_hull + [3] * (len(polys) - n_hull), dtype=np.int32)
    return np.array(polys), nv, np.array(normals), np.array(groups, dtype=np.int32), n_hull
