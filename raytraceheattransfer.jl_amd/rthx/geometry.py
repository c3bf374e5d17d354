"""Host-side 2D geometry: ``PolyVolume2D`` and the quad / triangle mesher.

Restates, on the host, the parts of the reference's data model that define
the exchange-factor index space:

* ``PolyVolume2D`` constructors — src/Domains/domains/PolyVolume2D.jl:2-184
  (vertex-mean midpoint :9/:103, signed shoelace ``volume`` :20-21/:112,
  wall lengths :23/:114) and ``calculateInwardNormal``
  (src/Domains/domains/calculateInwardNormal.jl:1-12);
* ``mesh_quad`` — ``meshQuad(volume, Nx, Ny)``, src/Meshing/meshing/meshQuad.jl:75-182,
  including its wall-solidity quirk (wall 2 only via ``elseif n == Nx``,
  wall 3 only via ``elseif m == Ny``, :145-161);
* ``mesh_triangle`` — ``meshTriangle(face, N)``, src/Meshing/meshing/meshTriangle.jl:2-103.

Sub-volumes inherit the parent's extinction (inheritVolumeProperty!,
src/Meshing/meshing/inheritVolumeProperty.jl:2-22) and, for solid walls that
lie on a parent edge, the parent's wall properties (addSubVolume.jl:21-35).
Nothing here runs on the GPU; this is input construction.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple, Union

import numpy as np

Number = Union[float, int]
Spectral = Union[float, Sequence[float]]


def _inward_normal(p1, p2, mid) -> Tuple[float, float]:
    """calculateInwardNormal.jl:1-12 (2D)."""
    ex, ey = p2[0] - p1[0], p2[1] - p1[1]
    nx, ny = ey, -ex
    norm = math.hypot(nx, ny)
    nx, ny = nx / norm, ny / norm
    wmx, wmy = (p1[0] + p2[0]) / 2, (p1[1] + p2[1]) / 2
    if nx * (wmx - mid[0]) + ny * (wmy - mid[1]) < 0:
        nx, ny = -nx, -ny
    return (nx, ny)


def _as_bins(v: Spectral, n_bins: int):
    if n_bins == 1 and np.isscalar(v):
        return float(v)
    arr = np.asarray(v, dtype=np.float64)
    if arr.ndim == 0:
        return np.full(n_bins, float(arr))
    return arr.copy()


class PolyVolume2D:
    """A 2D polygon (3 or 4 vertices) with gas and wall properties.

    Mirrors ``PolyVolume2D{Float64}(vertices, solidWalls, n_spectral_bins,
    kappa, sigma_s)`` (PolyVolume2D.jl:2-4, :96-98).  Grey faces hold scalar
    ``kappa_g`` / ``sigma_s_g``; spectral faces hold length-``n_bins`` arrays.
    """

    def __init__(self, vertices: Sequence[Tuple[Number, Number]], solid_walls: Sequence[bool],
                 n_spectral_bins: int = 1, kappa: Spectral = 0.0, sigma_s: Spectral = 0.0):
        n = len(vertices)
        if n not in (3, 4):
            raise ValueError("Only triangles and quadrilaterals are supported.")
        if len(solid_walls) != n:
            raise ValueError("solid_walls must have one entry per wall")
        self.vertices = [(float(x), float(y)) for x, y in vertices]
        self.solidWalls = [bool(b) for b in solid_walls]
        v = self.vertices
        if n == 4:
            self.midPoint = ((v[0][0] + v[1][0] + v[2][0] + v[3][0]) / 4,
                             (v[0][1] + v[1][1] + v[2][1] + v[3][1]) / 4)
            p = v
            self.volume = (0.5 * (p[0][0] * (p[1][1] - p[2][1]) + p[1][0] * (p[2][1] - p[0][1])
                                  + p[2][0] * (p[0][1] - p[1][1]))
                           + 0.5 * (p[2][0] * (p[3][1] - p[0][1]) + p[3][0] * (p[0][1] - p[2][1])
                                    + p[0][0] * (p[2][1] - p[3][1])))
        else:
            self.midPoint = ((v[0][0] + v[1][0] + v[2][0]) / 3, (v[0][1] + v[1][1] + v[2][1]) / 3)
            p = v
            self.volume = 0.5 * (p[0][0] * (p[1][1] - p[2][1]) + p[1][0] * (p[2][1] - p[0][1])
                                 + p[2][0] * (p[0][1] - p[1][1]))
        self.wallMidPoints = [((v[i][0] + v[(i + 1) % n][0]) / 2, (v[i][1] + v[(i + 1) % n][1]) / 2)
                              for i in range(n)]
        self.inwardNormals = [_inward_normal(v[i], v[(i + 1) % n], self.midPoint) for i in range(n)]
        self.area = [math.hypot(v[i][0] - v[(i + 1) % n][0], v[i][1] - v[(i + 1) % n][1])
                     for i in range(n)]
        self.n_bins = int(n_spectral_bins)
        self.kappa_g = _as_bins(kappa, self.n_bins)
        self.sigma_s_g = _as_bins(sigma_s, self.n_bins)
        zero = 0.0 if self.n_bins == 1 else np.zeros(self.n_bins)
        self.epsilon = [zero if np.isscalar(zero) else zero.copy() for _ in range(n)]
        self.T_in_w = [0.0] * n
        self.q_in_w = [0.0] * n
        self.T_in_g = 0.0
        self.q_in_g = 0.0
        self.T_g = 0.0
        self.T_w = [0.0] * n
        self.subVolumes: List["PolyVolume2D"] = []

    @property
    def n(self) -> int:
        return len(self.vertices)

    def beta(self, b: int = 0) -> float:
        """kappa_g[b] + sigma_s_g[b] (0-based bin)."""
        if np.isscalar(self.kappa_g):
            return float(self.kappa_g) + float(self.sigma_s_g)
        return float(self.kappa_g[b]) + float(self.sigma_s_g[b])

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"PolyVolume2D({self.vertices}, solid={self.solidWalls})"


def _containing_edge(sup: PolyVolume2D, p) -> Tuple[int, float]:
    """containing_edge, addSubVolume.jl:43-57."""
    best_d, best_k = math.inf, 0
    n = sup.n
    for k in range(n):
        a = sup.vertices[k]
        b = sup.vertices[(k + 1) % n]
        abx, aby = b[0] - a[0], b[1] - a[1]
        t = ((p[0] - a[0]) * abx + (p[1] - a[1]) * aby) / (abx * abx + aby * aby)
        t = min(max(t, 0.0), 1.0)
        d = math.hypot(p[0] - (a[0] + t * abx), p[1] - (a[1] + t * aby))
        if d < best_d:
            best_d, best_k = d, k
    return best_k, best_d


def _copy_prop(v):
    return v.copy() if isinstance(v, np.ndarray) else v


def add_sub_volume(sup: PolyVolume2D, sub: PolyVolume2D) -> None:
    """addSubVolume!, addSubVolume.jl:2-40 (inherit gas and solid-wall properties)."""
    sub.kappa_g = _copy_prop(sup.kappa_g)
    sub.sigma_s_g = _copy_prop(sup.sigma_s_g)
    sub.T_in_g = sup.T_in_g
    sub.q_in_g = sup.q_in_g * sub.volume / sup.volume if sup.volume != 0 else 0.0
    charlen = max(sup.area)
    for i in range(sub.n):
        if not sub.solidWalls[i]:
            continue
        m = sub.wallMidPoints[i]
        k, d = _containing_edge(sup, m)
        if d < 1e-8 * charlen and sup.solidWalls[k]:
            sub.epsilon[i] = _copy_prop(sup.epsilon[k])
            sub.T_in_w[i] = sup.T_in_w[k]
            sub.q_in_w[i] = sup.q_in_w[k] * sub.area[i] / sup.area[k] if sup.area[k] else 0.0
    sup.subVolumes.append(sub)


def mesh_quad(volume: PolyVolume2D, Nx: int, Ny: int) -> PolyVolume2D:
    """meshQuad(volume, Nx, Ny), meshQuad.jl:75-182.

    Fine cells are produced x-fastest then y (:139-179) and walls are numbered
    1 bottom, 2 right, 3 top, 4 left (here 0..3).
    """
    if volume.n != 4:
        raise ValueError("mesh_quad needs a quadrilateral")
    A, B, Cp, D = volume.vertices
    xs = (A[0], B[0], Cp[0], D[0], A[0])
    ys = (A[1], B[1], Cp[1], D[1], A[1])
    dXbot = xs[1] - xs[0]
    dXtop = xs[3] - xs[2]
    dXleft = xs[4] - xs[3]
    dYbot = ys[0] - ys[1]
    dYright = ys[1] - ys[2]
    dYleft = ys[3] - ys[0]
    xP = [[0.0] * (Ny + 1) for _ in range(Nx + 1)]
    yP = [[0.0] * (Ny + 1) for _ in range(Nx + 1)]
    for m in range(1, Ny + 2):
        rXleft = (m - 1) * dXleft / Ny
        rXright = dXbot - (m - 1) * (dXbot + dXtop) / Ny
        for n in range(1, Nx + 2):
            rYdown = (n - 1) * dYbot / Nx
            rYup = dYleft - (n - 1) * (dYleft + dYright) / Nx
            xP[n - 1][m - 1] = xs[0] - rXleft + (n - 1) * rXright / Nx
            yP[n - 1][m - 1] = ys[0] - rYdown + (m - 1) * rYup / Ny
    n_bins = volume.n_bins
    kd = volume.kappa_g if np.isscalar(volume.kappa_g) else volume.kappa_g[0]
    sd = volume.sigma_s_g if np.isscalar(volume.sigma_s_g) else volume.sigma_s_g[0]
    for m in range(1, Ny + 1):
        solid = [False, False, False, False]
        if m == 1:
            solid[0] = volume.solidWalls[0]
        elif m == Ny:
            solid[2] = volume.solidWalls[2]
        for n in range(1, Nx + 1):
            solid = [solid[0], False, solid[2], False]
            if n == 1:
                solid[3] = volume.solidWalls[3]
            elif n == Nx:
                solid[1] = volume.solidWalls[1]
            pts = [(xP[n - 1][m - 1], yP[n - 1][m - 1]), (xP[n][m - 1], yP[n][m - 1]),
                   (xP[n][m], yP[n][m]), (xP[n - 1][m], yP[n - 1][m])]
            sub = PolyVolume2D(pts, list(solid), n_bins, kd, sd)
            add_sub_volume(volume, sub)
    return volume


def mesh_triangle(face: PolyVolume2D, Ndim: int) -> PolyVolume2D:
    """meshTriangle(face, Ndim), meshTriangle.jl:2-103.

    The triangle is mirrored across its longest edge into a parallelogram,
    meshed as a quad, and the sub-cells on the triangle's side are kept; cells
    cut by the diagonal become triangles.  (N, N) gives N(N+1)/2 cells.
    """
    if face.n != 3:
        raise ValueError("mesh_triangle needs a triangle")
    n_bins = face.n_bins
    kd = face.kappa_g if np.isscalar(face.kappa_g) else face.kappa_g[0]
    sd = face.sigma_s_g if np.isscalar(face.sigma_s_g) else face.sigma_s_g[0]
    tri_mid = face.midPoint
    v = face.vertices
    norms = [math.hypot(v[0][0] - v[1][0], v[0][1] - v[1][1]),
             math.hypot(v[1][0] - v[2][0], v[1][1] - v[2][1]),
             math.hypot(v[2][0] - v[0][0], v[2][1] - v[0][1])]
    max_index = int(np.argmax(norms)) + 1  # findmax: first maximum, 1-based
    if max_index == 1:
        to_mirror, start = v[2], v[0]
        line = (v[1][0] - v[0][0], v[1][1] - v[0][1])
        diag_ind, mirror_ind = 1, 2
    elif max_index == 2:
        to_mirror, start = v[0], v[1]
        line = (v[2][0] - v[1][0], v[2][1] - v[1][1])
        diag_ind, mirror_ind = 2, 3
    else:
        to_mirror, start = v[1], v[2]
        line = (v[0][0] - v[2][0], v[0][1] - v[2][1])
        diag_ind, mirror_ind = 3, 4
    lmid = (start[0] + line[0] / 2, start[1] + line[1] / 2)
    vec = (to_mirror[0] - lmid[0], to_mirror[1] - lmid[1])
    mirrored = (-vec[0] + lmid[0], -vec[1] + lmid[1])
    s = face.solidWalls
    if max_index == 1:
        new_pts = [v[0], mirrored, v[1], v[2]]
        new_solid = [s[0], s[0], s[1], s[2]]
    elif max_index == 2:
        new_pts = [v[0], v[1], mirrored, v[2]]
        new_solid = [s[0], s[1], s[1], s[2]]
    else:
        new_pts = [v[0], v[1], v[2], mirrored]
        new_solid = [s[0], s[1], s[2], s[2]]
    tria_ids = [i for i in (1, 2, 3, 4) if i != mirror_ind]
    face2 = PolyVolume2D(new_pts, new_solid, n_bins, kd, sd)
    face2.kappa_g = _copy_prop(face.kappa_g)
    face2.sigma_s_g = _copy_prop(face.sigma_s_g)
    mesh_quad(face2, Ndim, Ndim)
    pv = (tri_mid[0] - start[0], tri_mid[1] - start[1])
    t = (pv[0] * line[0] + pv[1] * line[1]) / (line[0] * line[0] + line[1] * line[1])
    t = min(max(t, 0.0), 1.0)
    nearest = (start[0] + t * line[0], start[1] + t * line[1])
    for sub in face2.subVolumes:
        a = (tri_mid[0] - nearest[0], tri_mid[1] - nearest[1])
        b = (sub.midPoint[0] - nearest[0], sub.midPoint[1] - nearest[1])
        cos_sub = a[0] * b[0] + a[1] * b[1]
        if abs(cos_sub - 0.0) <= 1e-6:  # isapprox(x, 0.0, atol=1e-6)
            sub_ids = [i for i in (1, 2, 3, 4) if i not in (mirror_ind - 1, mirror_ind)]
            walls_ids = sorted(sub_ids + [diag_ind])
            walls_solid = [face.solidWalls[diag_ind - 1] if i == diag_ind else sub.solidWalls[i - 1]
                           for i in walls_ids]
            pts = [sub.vertices[i - 1] for i in tria_ids]
            keeper = PolyVolume2D(pts, walls_solid, n_bins, kd, sd)
            add_sub_volume(face, keeper)
        else:
            cos_d = b[0] * a[0] + b[1] * a[1]
            if cos_d > 0.0 - 1e-6:
                add_sub_volume(face, sub)
    return face
