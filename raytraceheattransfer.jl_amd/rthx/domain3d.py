"""3D surface enclosures: ViewFactorDomain3D on the MI355X.

Host mirror of ViewFactorDomain3D (src/Domains/domains/ViewFactorDomain3D.jl:2-101),
PolyFace3D (PolyFace3D.jl:2-45) and meshFaces (src/Meshing/meshing/meshFaces.jl,
projectPlane.jl, meshQuad.jl:2-73).  Calling the domain, ``domain3D()``
(ViewFactorDomain3D.jl:92-101), computes F_raw with the analytic view factors of
enclosureViewFactors3D on the device (rthx_view_factors_3d) and F_smooth with
the device smoothing (rthx_smooth_F, surfaces only, weights = areas).  No CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import List, Optional, Sequence

import numpy as np

from . import abi


def _unit(v):
    return v / np.linalg.norm(v)


def calculate_inward_normal_3d(p1, p2, p3, midpoint):
    """calculateInwardNormal.jl:14-25: the face normal flipped toward the
    domain midpoint."""
    n = _unit(np.cross(p2 - p1, p3 - p1))
    face_mid = (p1 + p2 + p3) / 3
    if np.dot(n, midpoint - face_mid) < 0:
        n = -n
    return n


class PolyFace3D:
    """PolyFace3D (PolyFace3D.jl:2-45, DomainStructs.jl:132-156)."""

    def __init__(self, vertices: Sequence, solid: bool, domain_midpoint, epsilon, q_in_w: float, T_in_w: float):
        self.vertices = [np.asarray(v, dtype=np.float64) for v in vertices]
        v = self.vertices
        self.solidFace = bool(solid)
        self.midPoint = sum(v) / len(v)
        if len(v) == 3:
            self.area = float(np.linalg.norm(np.cross(v[1] - v[0], v[2] - v[0])) / 2)
        else:
            self.area = float(np.linalg.norm(np.cross(v[1] - v[0], v[3] - v[0])))
        self.inwardNormal = calculate_inward_normal_3d(v[0], v[1], v[2], domain_midpoint)
        self.subFaces: Optional[List["PolyFace3D"]] = None
        self.epsilon = epsilon
        spectral = isinstance(epsilon, (list, np.ndarray))
        nb = len(epsilon) if spectral else 0
        for name in ("j_w", "g_a_w", "e_w", "r_w", "g_w", "i_w"):
            setattr(self, name, np.zeros(nb) if spectral else None)
        self.q_in_w = float(q_in_w)
        self.q_w = None
        self.T_in_w = float(T_in_w)
        self.T_w = None


# --- meshFaces (src/Meshing/meshing/) --------------------------------------
def _quat_to_rot(q):
    w, x, y, z = q
    return np.array([[1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * z * w, 2 * x * z + 2 * y * w],
                     [2 * x * y + 2 * z * w, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * x * w],
                     [2 * x * z - 2 * y * w, 2 * y * z + 2 * x * w, 1 - 2 * x * x - 2 * y * y]])


def _project_plane_flat(pts):
    """projectPlaneFlat (projectPlane.jl:3-36): rotation taking the face normal
    to +z (quaternion form) and the translation moving vertex 1 to the origin."""
    n = _unit(np.cross(pts[1] - pts[0], pts[2] - pts[0]))
    z = np.array([0.0, 0.0, 1.0])
    axis = np.cross(n, z)
    angle = math.acos(min(max(float(np.dot(n, z)), -1.0), 1.0))
    if np.linalg.norm(axis) < 1e-10:
        R = np.eye(3) if np.dot(n, z) > 0 else np.diag([1.0, 1.0, -1.0])
    else:
        axis = _unit(axis)
        R = _quat_to_rot(np.r_[math.cos(angle / 2), math.sin(angle / 2) * axis])
    return R, -pts[0]


def _mesh_quad_flat(face, Nx, Ny):
    """meshQuad(face::Vector{Vector}, Nx, Ny) (meshQuad.jl:2-73): the flat quad
    split into Nx x Ny cells (x fastest), as (p1, p2, p3, p4) lists."""
    xs = [face[0][0], face[1][0], face[2][0], face[3][0], face[0][0]]
    ys = [face[0][1], face[1][1], face[2][1], face[3][1], face[0][1]]
    dXbot, dXtop, dXleft = xs[1] - xs[0], xs[3] - xs[2], xs[4] - xs[3]
    dYbot, dYright, dYleft = ys[0] - ys[1], ys[1] - ys[2], ys[3] - ys[0]
    X = np.zeros((Nx + 1, Ny + 1))
    Y = np.zeros((Nx + 1, Ny + 1))
    for m in range(Ny + 1):
        mvl = m * dXleft / Ny
        mvr = dXbot - m * (dXbot + dXtop) / Ny
        for k in range(Nx + 1):
            mvd = k * dYbot / Nx
            mvu = dYleft - k * (dYleft + dYright) / Nx
            X[k, m] = xs[0] - mvl + k * mvr / Nx
            Y[k, m] = ys[0] - mvd + m * mvu / Ny
    out = ([], [], [], [])
    for m in range(Ny):
        for k in range(Nx):
            out[0].append(np.array([X[k, m], Y[k, m], 0.0]))
            out[1].append(np.array([X[k + 1, m], Y[k + 1, m], 0.0]))
            out[2].append(np.array([X[k + 1, m + 1], Y[k + 1, m + 1], 0.0]))
            out[3].append(np.array([X[k, m + 1], Y[k, m + 1], 0.0]))
    return out


def _mesh_triangle_flat(face, Nx, Ny):
    """meshTriangle(face::Vector{Vector}, Nx, Ny) (meshTriangle.jl:106-220):
    the flat triangle is mirrored across its longest edge (first maximum of
    the three edge lengths) into a parallelogram, which is meshed as a quad
    (meshQuad.jl:75-182); cells whose midpoint lies on that edge (within
    1e-6) become triangles (the cell's corners other than the mirrored one's
    position, p4 = p3), cells on the triangle's side are kept, the others
    dropped.  Returns (p1, p2, p3, p4) lists of points with z = 0."""
    from .geometry import PolyVolume2D, mesh_quad

    P = [np.asarray(q, dtype=np.float64)[:2] for q in face]
    tri_mid = (np.asarray(face[0], dtype=np.float64) + np.asarray(face[1], dtype=np.float64)
               + np.asarray(face[2], dtype=np.float64))[:2] / 3
    norms = [np.linalg.norm(P[0] - P[1]), np.linalg.norm(P[1] - P[2]), np.linalg.norm(P[2] - P[0])]
    max_index = int(np.argmax(norms)) + 1  # findmax: first maximum, 1-based
    to_mirror, start = {1: (P[2], P[0]), 2: (P[0], P[1]), 3: (P[1], P[2])}[max_index]
    line = {1: P[1] - P[0], 2: P[2] - P[1], 3: P[0] - P[2]}[max_index]
    mirror_ind = max_index + 1
    lmid = start + line / 2
    mirrored = -(to_mirror - lmid) + lmid
    new_pts = [P[0], P[1], P[2]]
    new_pts.insert(mirror_ind - 1, mirrored)
    tria_ids = [i for i in (1, 2, 3, 4) if i != mirror_ind]
    face2 = PolyVolume2D([tuple(q) for q in new_pts], [True] * 4, 1, 1.0, 1.0)
    mesh_quad(face2, Nx, Ny)
    t = float(np.dot(tri_mid - start, line) / np.dot(line, line))
    nearest = start + min(max(t, 0.0), 1.0) * line
    out = ([], [], [], [])
    for sub in face2.subVolumes:
        cos_sub = float(np.dot(tri_mid - nearest, np.asarray(sub.midPoint) - nearest))
        if abs(cos_sub) <= 1e-6:  # isapprox(x, 0.0, atol=1e-6): cut by the diagonal
            kv = [sub.vertices[i - 1] for i in tria_ids]
            corners = (kv[0], kv[1], kv[2], kv[2])
        elif cos_sub > 0.0 - 1e-6:
            corners = tuple(sub.vertices)
        else:
            continue
        for k in range(4):
            out[k].append(np.array([corners[k][0], corners[k][1], 0.0]))
    return out


def mesh_faces(points: np.ndarray, faces: np.ndarray, Ndim: int):
    """meshFaces (meshFaces.jl:2-18): per face the sub-face corner lists
    (p1, p2, p3, p4), meshed in the face's own plane (meshQuad, or
    meshTriangle for triangles: N(N+1)/2 sub-faces) and projected back.
    (The reference sizes every face's list by face 1's sub-face count,
    ViewFactorDomain3D.jl:41; here each face keeps its own.)"""
    out = []
    for row in faces:
        pts = [np.asarray(points[i], dtype=np.float64) for i in row]
        R, T = _project_plane_flat(pts)
        flat = [R @ (p + T) for p in pts]
        cells = _mesh_triangle_flat(flat, Ndim, Ndim) if len(pts) == 3 else _mesh_quad_flat(flat, Ndim, Ndim)
        Rinv = np.linalg.inv(R)
        out.append(tuple([Rinv @ q - T for q in corner] for corner in cells))
    return out


class ViewFactorDomain3D:
    """ViewFactorDomain3D(points, faces, Ndims, q_in_w, T_in_w, epsilon)
    (ViewFactorDomain3D.jl:2-89).  ``faces`` holds 1-based vertex indices as in
    the reference."""

    def __init__(self, points, faces, Ndims: int, q_in_w, T_in_w, epsilon):
        points = np.asarray(points, dtype=np.float64)
        faces = np.asarray(faces, dtype=np.int64) - 1
        is_spectral = isinstance(epsilon[0], (list, np.ndarray))
        if is_spectral:
            spread = np.std([np.std(e) for e in epsilon])
            self.spectral_mode = "spectral_variable" if spread > 1e-6 else "spectral_uniform"
        else:
            self.spectral_mode = "grey"
        self.n_spectral_bins = len(epsilon[0]) if is_spectral else 1
        self.points, self.faces, self.Ndims = points, faces + 1, int(Ndims)
        mid = points.mean(axis=0)
        self.facesMesh: List[PolyFace3D] = []
        for i, row in enumerate(faces):
            self.facesMesh.append(PolyFace3D([points[j] for j in row], True, mid, epsilon[i], q_in_w[i], T_in_w[i]))
        mesh = mesh_faces(points, faces, Ndims)
        self.uniform_epsilon = True
        first = None
        for i, sf in enumerate(self.facesMesh):
            sf.subFaces = []
            p1, p2, p3, p4 = mesh[i]
            for k in range(len(p1)):
                tri = np.allclose(p3[k], p4[k], atol=1e-5, rtol=0)
                verts = [p1[k], p2[k], p3[k]] if tri else [p1[k], p2[k], p3[k], p4[k]]
                sf.subFaces.append(PolyFace3D(verts, True, mid, epsilon[i], 0.0, T_in_w[i]))
            total = sum(s.area for s in sf.subFaces)
            for s in sf.subFaces:  # flux distributed by area (:62-67)
                s.q_in_w = float(q_in_w[i]) * (s.area / total)
                e = np.atleast_1d(s.epsilon)
                if first is None:
                    first = e[0]
                elif np.any(np.abs(e - first) > 1e-5):
                    self.uniform_epsilon = False
        self.wavelength_band_limits = None
        self.energy_error = None
        self.surfaces_only = True
        n = self.num_elements
        self.F_raw = np.zeros((n, n))
        self.F_smooth = np.zeros((n, n))
        self.last_vf_info: dict = {}

    @property
    def num_elements(self) -> int:
        return sum(len(sf.subFaces) for sf in self.facesMesh)

    def subfaces(self) -> List[PolyFace3D]:
        return [s for sf in self.facesMesh for s in sf.subFaces]

    def polygon_arrays(self):
        """(xyz[n][4][3], nv[n]) of the sub-faces in enclosureViewFactors3D's
        linear order (face-major, fromLinear, enclosureViewFactors3D.jl:96-100)."""
        subs = self.subfaces()
        xyz = np.zeros((len(subs), 4, 3))
        nv = np.zeros(len(subs), dtype=np.int32)
        for k, s in enumerate(subs):
            nv[k] = len(s.vertices)
            xyz[k, : nv[k]] = np.array(s.vertices)
        return xyz, nv

    def __call__(self, parallel: bool = True, max_iters: int = 1000, device: int = 0, verbose: bool = False,
                 method: str = "analytic", rays_tot: int = 0, seed: int = 1):
        """ViewFactorDomain3D functor (ViewFactorDomain3D.jl:92-101) ->
        enclosureViewFactors3D (enclosureViewFactors3D.jl:1-94): F_raw on the
        device, sub-face areas from viewFactor3D's formulas, then smooth_F with
        smooth_surfaces_only = true.  ``method="montecarlo"`` (an extension:
        enclosures with obstructions) traces ``rays_tot`` rays instead
        (rthx.trace3d, rays leave along each sub-face's inward normal)."""
        from .smoothing import smooth_F

        xyz, nv = self.polygon_arrays()
        if method == "montecarlo":
            from .trace3d import exchange_factors_3d

            _, area, _ = view_factors_3d(xyz, nv, device=device, with_F=False)
            normals = np.array([s.inwardNormal for s in self.subfaces()])
            R = max(1, int(rays_tot) // len(nv))
            F_raw = exchange_factors_3d(xyz, nv, normals, R, seed=seed, device=device).toarray()
            info = {"rays_per_emitter": R}
        elif method == "analytic":
            F_raw, area, info = view_factors_3d(xyz, nv, device=device)
        else:
            raise ValueError(f"unknown method {method!r}: 'analytic' or 'montecarlo'")
        for s, a in zip(self.subfaces(), area):
            s.area = float(a)  # enclosureViewFactors3D.jl:48-49
        self.F_raw = F_raw
        self.F_smooth = smooth_F(F_raw, area, len(area), max_iters=max_iters, smooth_surfaces_only=True,
                                 verbose=verbose, device=device)
        if not isinstance(self.F_smooth, np.ndarray):
            self.F_smooth = self.F_smooth.toarray()
        self.last_vf_info = info
        return None


def view_factors_3d(xyz, nv, device: int = 0, with_F: bool = True):
    """rthx_view_factors_3d: (F[n, n], area[n], info); with_F=False computes
    the areas only (no device needed)."""
    from ._lib import check, load

    lib = load()
    x = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 12)
    k = np.ascontiguousarray(nv, dtype=np.int32)
    n = len(k)
    F = np.empty((n, n)) if with_F else None
    area = np.empty(n)
    a = abi.Vf3dArgs()
    a.device = device
    inf = abi.Vf3dInfo()
    check(lib.rthx_view_factors_3d(abi.ptr(x, C.c_double), abi.ptr(k, C.c_int32), n, C.byref(a),
                                   abi.ptr(F, C.c_double) if with_F else None, abi.ptr(area, C.c_double),
                                   C.byref(inf)))
    return F, area, inf.as_dict()
