"""Generate the committed golden fixtures (run in the build container only).

reference_tables.json — known answers transcribed from the reference's own
test files (parsed from /root/reference/test when it is present):
  * Crosbie & Schrenker (1984) centreline table, test/test_2d_grey.jl:25-33,
    tolerance test/test_2d_grey.jl:35 (rtol 0.05, norm-wise isapprox);
  * wedge centre limit ((T^4 + 0)/2)^(1/4) and its 2 K tolerance,
    test/test_triangle_mesh.jl:66-69;
  * Stefan-Boltzmann constant, src/RayTraceHeatTransfer.jl:20;
  * Philox-4x32-10 known-answer vectors (Random123 kat_vectors; the RNG
    is this build's, the reference's rand() is unseeded);
  * Hottel crossed-strings view factors of the unit square.

oracle_c1_seed1.npz — CPU-restatement absorber counts for README Ex.1
(11x11, kappa=1, 1e6 rays, seed 1): a regression fixture that the HIP path
must reproduce exactly.

reference_known_answers.json (`python tests/golden/make_golden.py known`) --
the diffusion limit, reflecting-wall energy and parallel-plate tests of the
reference and its icosphere-enclosure readme example (main_known_answers).

reference_3d.json (`python tests/golden/make_golden.py 3d`) — the 3D view
factor known answers of test/test_3d_viewfactors.jl (Narayanaswamy 2015
examples :31-75 and the EES unit-cube table :101-143, tolerance VF_TOLERANCE
:22, rotations :194-213) and the cube enclosure / tolerances of
test/test_3d_heat_transfer.jl:22-23,29-205.
"""
import json
import math
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def parse_julia_vector(text, name):
    m = re.search(name + r"\s*=\s*\[(.*?)\]", text, re.S)
    return [float(x) for x in m.group(1).replace("\n", " ").split(",") if x.strip()]


def main():
    ref = "/root/reference/test/test_2d_grey.jl"
    tables = {}
    if os.path.exists(ref):
        txt = open(ref).read()
        tables["crosbie_schrenker"] = {
            "source": "test/test_2d_grey.jl:25-33",
            "relative_tau_z": parse_julia_vector(txt, "RELATIVE_TAU_Z"),
            "source_func_center": parse_julia_vector(txt, "SOURCE_FUNC_CENTER"),
            "rtol": 0.05,
            "rtol_source": "test/test_2d_grey.jl:35 (isapprox on vectors: norm-wise)",
        }
    else:  # keep the committed values
        with open(os.path.join(HERE, "reference_tables.json")) as fh:
            tables = json.load(fh)
    tables["wedge_center_limit"] = {
        "source": "test/test_triangle_mesh.jl:48-74",
        "T_hot": 1000.0,
        "T_limit": ((1000.0 ** 4 + 0.0) / 2) ** 0.25,
        "tol_K": 2.0,
        "n_wedges": 16,
        "ndiv": 11,
        "rays": 10_000_000,
    }
    tables["stefan_boltzmann"] = {"source": "src/RayTraceHeatTransfer.jl:20", "value": 5.670374419e-8}
    tables["philox4x32_10_kat"] = {
        "source": "Random123 kat_vectors (Salmon et al. SC'11)",
        "vectors": [
            {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]},
            {"ctr": [0xFFFFFFFF] * 4, "key": [0xFFFFFFFF] * 2,
             "out": [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]},
            {"ctr": [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], "key": [0xA4093822, 0x299F31D0],
             "out": [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]},
        ],
    }
    tables["crossed_strings_unit_square"] = {
        "source": "Hottel crossed strings (SURVEY.md §8(c))",
        "adjacent": (2 - math.sqrt(2)) / 2,
        "opposite": math.sqrt(2) - 1,
    }
    with open(os.path.join(HERE, "reference_tables.json"), "w") as fh:
        json.dump(tables, fh, indent=1)

    import helpers as H
    from oracle import oracle
    from rthx import _lib

    dom = H.square_domain(11)
    flat = dom.flat()
    R = 1_000_000 // flat.n_emitters
    args, _k = _lib.make_args(0, R, H.NUDGE, 1, 0, flat.n_emitters)
    rp, cols, cnt, info, _ = oracle.trace_exchange(flat, args, 8)
    np.savez_compressed(os.path.join(HERE, "oracle_c1_seed1.npz"), row_ptr=rp, cols=cols, counts=cnt,
                        R=np.int64(R), seed=np.int64(1))
    print("wrote fixtures; C1 nnz", info["nnz"])


def parse_julia_matrix(body):
    rows = [r.strip() for r in body.replace("\n", " ").split(";") if r.strip()]
    return [[float(x) for x in r.split()] for r in rows]


def main_3d():
    ref = "/root/reference/test/test_3d_viewfactors.jl"
    txt = open(ref).read()
    cases = []
    for m in re.finditer(r'name = "([^"]+)",\s*poly_A = \[(.*?)\],\s*poly_B = \[(.*?)\],\s*F_ref = ([0-9.eE+-]+)',
                         txt, re.S):
        cases.append({"name": m.group(1), "poly_A": parse_julia_matrix(m.group(2)),
                      "poly_B": parse_julia_matrix(m.group(3)), "F_ref": float(m.group(4))})
    ees = re.search(r"F_EES = \[(.*?)\]", txt, re.S).group(1)
    points = re.search(r"points = \[(.*?)\]", txt, re.S).group(1)
    faces = re.search(r"faces = \[(.*?)\]", re.sub(r"#[^\n]*", "", txt), re.S).group(1)
    tol = float(re.search(r"VF_TOLERANCE = ([0-9.eE+-]+)", txt).group(1))
    rot = [(a, eval(ang.replace("π", "math.pi"))) for a, ang in
           re.findall(r"\(:(\w), (π/\d|π)[^)]*\)", txt.split("rotations = [")[1].split("]")[0])]
    ht = open("/root/reference/test/test_3d_heat_transfer.jl").read()
    out = {
        "source": "test/test_3d_viewfactors.jl, test/test_3d_heat_transfer.jl",
        "vf_tolerance": tol,
        "narayanaswamy": cases,
        "cube_points": parse_julia_matrix(points),
        "cube_faces": [[int(v) for v in r] for r in parse_julia_matrix(faces)],
        "F_EES": parse_julia_matrix(ees),
        "rotations": [{"axis": a, "angle": ang} for a, ang in rot],
        "temp_tolerance_K": float(re.search(r"TEMP_TOLERANCE = ([0-9.eE+-]+)", ht).group(1)),
        "energy_tolerance_W": float(re.search(r"ENERGY_TOLERANCE = ([0-9.eE+-]+)", ht).group(1)),
    }
    with open(os.path.join(HERE, "reference_3d.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote reference_3d.json:", len(cases), "Narayanaswamy cases,", len(rot), "rotations")


def _num(txt, pattern):
    return float(re.search(pattern, txt, re.S).group(1).replace("_", ""))


def main_known_answers():
    """reference_known_answers.json (`python tests/golden/make_golden.py known`):
    the remaining known answers of the reference's own tests and readme, parsed
    from the files (constants, tolerances, geometry); the tests restate the
    reference's formulas around them.
      * diffusion limit: test/test_2d_diffusion.jl:15-77;
      * reflecting-wall energy conservation: test/test_2d_grey_reflecting.jl:42-69;
      * parallel plates vs the textbook flux: test/test_2d_grey_reflecting.jl:85-137;
      * the icosphere enclosure's equator limit: readme.md:532-704 (icosahedron
        vertices and faces of icosphere_mesh, n_cap, Ndim, the level table)."""
    ref = "/root/reference"
    dif = open(os.path.join(ref, "test/test_2d_diffusion.jl")).read()
    refl = open(os.path.join(ref, "test/test_2d_grey_reflecting.jl")).read()
    readme = open(os.path.join(ref, "readme.md")).read()
    out = {"source": "test/test_2d_diffusion.jl, test/test_2d_grey_reflecting.jl, readme.md:532-704"}
    n_side = int(re.search(r'\("sparse", (\d+), true\)', dif).group(1))
    out["diffusion"] = {
        "source": "test/test_2d_diffusion.jl:15-77",
        "T_hot": _num(dif, r"T_HOT_DIFF\s*=\s*([0-9.]+)"),
        "beta": _num(dif, r"BETA_DIFF\s*=\s*([0-9.]+)"),
        "aspect": _num(dif, r"ASPECT_DIFF\s*=\s*([0-9.]+)"),
        "N_side": n_side,
        "rays_per_element": int(_num(dif, r"N_rays = \(4 \* N_side \+ N_side\^2\) \* ([0-9_]+)")),
        "rms_tol": _num(dif, r"RMS_TOL\s*=\s*([0-9.]+)"),
        "ratio_tol": _num(dif, r"RATIO_TOL\s*=\s*([0-9.]+)"),
        "energy_tol": _num(dif, r"abs\(sum\(mesh.energy_error\)\) < ([0-9.eE+-]+)"),
        "expect_sparse": True,
        "formula": "diffusion_S(z) = E_b1 - (3 beta z / 4) q_z, q_z = (E_bw1 - E_bw2) / (3 beta D / 4 + 1/eps1 "
                   "+ 1/eps2 - 1), E_b1 = E_bw1 + q_z (1/2 - 1/eps1); D = eps = E_bw1 = 1, E_bw2 = 0 (:19-23,:46)",
    }
    t1 = refl.split("TEST 2")[0]
    t2 = refl.split("TEST 2")[1]
    out["reflecting_energy"] = {
        "source": "test/test_2d_grey_reflecting.jl:42-69",
        "T_hot": _num(t1, r"T_hot\s*=\s*([0-9.]+)"),
        "Ndim": int(_num(t1, r"Ndim\s*=\s*([0-9]+)")),
        "rays": int(_num(t1, r"N_rays_total = ([0-9_]+)")),
        "kappa": 1.0,
        "T_in_w": [1000.0, -1.0, -1.0, -1.0],
        "epsilon": [float(x) for x in re.search(r"face.epsilon = \[([^\]]+)\]", t1).group(1).split(",")],
        "energy_tol": _num(refl, r"ENERGY_TOLERANCE = ([0-9.eE+-]+)"),
    }
    out["parallel_plates"] = {
        "source": "test/test_2d_grey_reflecting.jl:85-137",
        "eps": _num(t2, r"eps_plates = ([0-9.]+)"),
        "T_hot": _num(t2, r"T_hot\s*=\s*([0-9.]+)"),
        "T_cold": _num(t2, r"T_cold\s*=\s*([0-9.]+)"),
        "W": _num(t2, r"W = ([0-9.]+)"),
        "H": _num(t2, r"H = ([0-9.]+)"),
        "Nx": int(_num(t2, r"Nx = ([0-9]+)")),
        "Ny": int(_num(t2, r"Ny = ([0-9]+)")),
        "rays": int(_num(t2, r"N_rays_total = ([0-9_]+)")),
        "kappa": _num(t2, r"PolyVolume2D\{Float64\}\(vertices, solidWalls, 1, ([0-9.eE+-]+), 0.0\)"),
        "k_dykstra": int(_num(t2, r"k_dykstra=([0-9]+)")),
        "rel_tol": _num(refl, r"ANALYTICAL_TOLERANCE = ([0-9.]+)"),
        "energy_tol": _num(refl, r"ENERGY_TOLERANCE = ([0-9.eE+-]+)"),
        "formula": "q = sigma (T_hot^4 - T_cold^4) / (1/eps + 1/eps - 1), mean over the central Nx div 5 "
                   "bottom-wall elements (:118-136)",
    }
    ico = readme[readme.index("function icosphere_mesh"):]
    raw = re.search(r"ico_points_raw = \[(.*?)\]", ico, re.S).group(1)
    vals = [x for x in re.split(r"[\s;]+", raw.strip()) if x]
    phi = (1 + math.sqrt(5)) / 2
    nums = [phi if v == "φ" else -phi if v == "-φ" else float(v) for v in vals]
    faces = re.search(r"faces = \[(.*?)\]", ico, re.S).group(1)
    fnums = [int(x) for x in re.split(r"[\s;]+", faces.strip()) if x]
    table = re.findall(r"\|\s*(\d)\s*\|\s*(\d+)\s*\|\s*([0-9.eE+-]+)\s*\|", readme[readme.index("T_equator"):])
    out["icosphere"] = {
        "source": "readme.md:532-704",
        "ico_points_raw": [nums[i:i + 3] for i in range(0, len(nums), 3)],
        "faces": [fnums[i:i + 3] for i in range(0, len(fnums), 3)],
        "n_cap": int(_num(ico, r"n_cap\s*=\s*([0-9]+)")),
        "Ndim": 1,
        "T_hot": _num(ico, r"T_hot\s*=\s*([0-9.]+)"),
        "T_cold": _num(ico, r"T_cold\s*=\s*([0-9.]+)"),
        "T_limit": ((1000.0 ** 4 + 0.0 ** 4) / 2) ** 0.25,
        "analytic_error_K": {lvl: float(err) for lvl, _ntri, err in table},
    }
    assert len(out["icosphere"]["ico_points_raw"]) == 12 and len(out["icosphere"]["faces"]) == 20
    with open(os.path.join(HERE, "reference_known_answers.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote reference_known_answers.json")


if __name__ == "__main__":
    if sys.argv[1:] == ["3d"]:
        main_3d()
    elif sys.argv[1:] == ["known"]:
        main_known_answers()
    else:
        main()
