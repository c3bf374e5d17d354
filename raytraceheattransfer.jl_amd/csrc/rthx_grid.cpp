// rthx_grid.cpp — host-side builder of the device point-location grid.
//
// The reference locates a point with a uniform grid (cell size 2*sqrt(mean
// area), spatialAccelerations.jl:2-59) whose cells list every polygon whose
// bbox meets the cell; candidates are tested in ascending order with the
// crossing-number test until the first hit (findFace2D.jl:2-27, :77-101).
// On a GPU that loop is the largest divergent cost of a ray.
//
// The device grid answers the same question with one record per cell: the
// polygon edges that cross a cell (at most two distinct lines for cells of
// half a polygon in a mesh of convex cells) split it into regions, and each
// region is verified -- by exact polygon clipping -- to lie inside exactly one
// polygon (or outside all of them).  A lookup is then two line tests and a
// table read, the same for every lane.  Cells that do not fit (a vertex
// where three or more edges meet, non-convex polygons) keep the candidate
// list, ordered by overlap area, and run the point-in-polygon loop.
// Decisions differ from the reference only for points within rounding of an
// edge, where the reference's own answer depends on the candidate order.
#include "rthx_grid.h"

#include <algorithm>
#include <cmath>

namespace rthx {
namespace {

struct P2 {
  double x, y;
};
using Poly = std::vector<P2>;

double area(const Poly& p) {
  double A = 0.0;
  for (size_t i = 0; i < p.size(); ++i) {
    const P2& a = p[i];
    const P2& b = p[(i + 1) % p.size()];
    A += a.x * b.y - b.x * a.y;
  }
  return 0.5 * A;
}

// keep a x + b y + c >= 0
Poly clip_half(const Poly& in, double a, double b, double c) {
  Poly out;
  const size_t n = in.size();
  for (size_t i = 0; i < n; ++i) {
    const P2& p = in[i];
    const P2& q = in[(i + 1) % n];
    double sp = a * p.x + b * p.y + c, sq = a * q.x + b * q.y + c;
    if (sp >= 0) out.push_back(p);
    if ((sp >= 0) != (sq >= 0)) {
      double t = sp / (sp - sq);
      out.push_back({p.x + t * (q.x - p.x), p.y + t * (q.y - p.y)});
    }
  }
  return out;
}

Poly rect(double x0, double x1, double y0, double y1) { return {{x0, y0}, {x1, y0}, {x1, y1}, {x0, y1}}; }

struct Line {
  double a, b, c;
};

// interior half-planes of a convex polygon (orientation-independent)
bool convex_halfplanes(const double* v, int n, std::vector<Line>& hp) {
  double A = 0.0;
  for (int i = 0; i < n; ++i) {
    int j = (i + 1) % n;
    A += v[2 * i] * v[2 * j + 1] - v[2 * j] * v[2 * i + 1];
  }
  double sgn = A > 0 ? 1.0 : -1.0;
  int pos = 0, neg = 0;
  for (int i = 0; i < n; ++i) {
    int j = (i + 1) % n, k = (i + 2) % n;
    double cr = (v[2 * j] - v[2 * i]) * (v[2 * k + 1] - v[2 * j + 1]) - (v[2 * j + 1] - v[2 * i + 1]) * (v[2 * k] - v[2 * j]);
    pos += cr > 0;
    neg += cr < 0;
  }
  if (pos && neg) return false;
  hp.clear();
  for (int i = 0; i < n; ++i) {
    int j = (i + 1) % n;
    double ex = v[2 * j] - v[2 * i], ey = v[2 * j + 1] - v[2 * i + 1];
    double len = std::sqrt(ex * ex + ey * ey);
    if (len == 0) return false;
    double a = -sgn * ey / len, b = sgn * ex / len;
    hp.push_back({a, b, -(a * v[2 * i] + b * v[2 * i + 1])});
  }
  return true;
}

Poly clip_convex(Poly p, const std::vector<Line>& hp) {
  for (const Line& l : hp) {
    if (p.empty()) break;
    p = clip_half(p, l.a, l.b, l.c);
  }
  return p;
}

// Liang-Barsky: length of segment (p, q) inside [x0,x1]x[y0,y1]
double seg_len_in_rect(P2 p, P2 q, double x0, double x1, double y0, double y1) {
  double t0 = 0.0, t1 = 1.0, dx = q.x - p.x, dy = q.y - p.y;
  double pp[4] = {-dx, dx, -dy, dy};
  double qq[4] = {p.x - x0, x1 - p.x, p.y - y0, y1 - p.y};
  for (int i = 0; i < 4; ++i) {
    if (pp[i] == 0) {
      if (qq[i] < 0) return 0.0;
    } else {
      double t = qq[i] / pp[i];
      if (pp[i] < 0) t0 = std::max(t0, t);
      else t1 = std::min(t1, t);
    }
  }
  if (t1 <= t0) return 0.0;
  return (t1 - t0) * std::sqrt(dx * dx + dy * dy);
}

}  // namespace

GridBuild build_cell_grid(const int32_t* nv, const double* xy, int first, int count, double cells_per_extent,
                          std::vector<CellRec>& cells, std::vector<int32_t>& lists, std::vector<int32_t>& items) {
  GridBuild G{};
  double minx = INFINITY, maxx = -INFINITY, miny = INFINITY, maxy = -INFINITY, sw = 0.0, sh = 0.0;
  std::vector<double> bb(4 * (size_t)count);
  for (int f = 0; f < count; ++f) {
    const double* v = xy + 8 * (size_t)(first + f);
    double a = INFINITY, b = -INFINITY, c = INFINITY, d = -INFINITY;
    for (int i = 0; i < nv[first + f]; ++i) {
      a = std::min(a, v[2 * i]); b = std::max(b, v[2 * i]);
      c = std::min(c, v[2 * i + 1]); d = std::max(d, v[2 * i + 1]);
    }
    bb[4 * f] = a; bb[4 * f + 1] = b; bb[4 * f + 2] = c; bb[4 * f + 3] = d;
    minx = std::min(minx, a); maxx = std::max(maxx, b); miny = std::min(miny, c); maxy = std::max(maxy, d);
    sw += b - a;
    sh += d - c;
  }
  const double ext = std::max(maxx - minx, maxy - miny);
  double sx = std::max(sw / count / cells_per_extent, 1e-9 * ext);
  double sy = std::max(sh / count / cells_per_extent, 1e-9 * ext);
  double nxd, nyd;
  auto dims = [&]() {
    nxd = std::max(1.0, std::ceil((maxx - minx) / sx + 0.02));
    nyd = std::max(1.0, std::ceil((maxy - miny) / sy + 0.02));
  };
  dims();
  const double cap = std::max(64.0, 64.0 * count);
  if (nxd * nyd > cap) {
    double k = std::sqrt(nxd * nyd / cap);
    sx *= k;
    sy *= k;
    dims();
  }
  G.nx = (int32_t)nxd;
  G.ny = (int32_t)nyd;
  // pad so that polygon edges of a regular mesh do not sit on cell lines
  G.ox = minx - 0.01 * sx;
  G.oy = miny - 0.01 * sy;
  G.inv_x = 1.0 / sx;
  G.inv_y = 1.0 / sy;
  const int64_t ncell = (int64_t)G.nx * G.ny;

  // candidates per cell: every polygon whose bbox meets the cell, with the
  // area of the polygon inside the cell
  struct Cand {
    int64_t cell;
    int32_t f;
    double area;
  };
  std::vector<Cand> cand;
  cand.reserve((size_t)count * 8);
  std::vector<std::vector<Line>> hps(count);
  std::vector<char> convex(count);
  for (int f = 0; f < count; ++f) {
    const double* v = xy + 8 * (size_t)(first + f);
    convex[f] = convex_halfplanes(v, nv[first + f], hps[f]);
    int64_t i0 = (int64_t)std::floor((bb[4 * f] - G.ox) * G.inv_x);
    int64_t i1 = (int64_t)std::floor((bb[4 * f + 1] - G.ox) * G.inv_x);
    int64_t j0 = (int64_t)std::floor((bb[4 * f + 2] - G.oy) * G.inv_y);
    int64_t j1 = (int64_t)std::floor((bb[4 * f + 3] - G.oy) * G.inv_y);
    i0 = std::max<int64_t>(0, i0); j0 = std::max<int64_t>(0, j0);
    i1 = std::min<int64_t>(G.nx - 1, i1); j1 = std::min<int64_t>(G.ny - 1, j1);
    Poly pf;
    for (int i = 0; i < nv[first + f]; ++i) pf.push_back({v[2 * i], v[2 * i + 1]});
    if (area(pf) < 0) std::reverse(pf.begin(), pf.end());
    for (int64_t j = j0; j <= j1; ++j)
      for (int64_t i = i0; i <= i1; ++i) {
        double x0 = G.ox + i * sx, y0 = G.oy + j * sy;
        // area of polygon f inside the cell (clip the polygon by the cell's 4 half-planes)
        Poly q = clip_half(pf, 1, 0, -x0);
        q = clip_half(q, -1, 0, x0 + sx);
        q = clip_half(q, 0, 1, -y0);
        q = clip_half(q, 0, -1, y0 + sy);
        double A = q.size() >= 3 ? std::fabs(area(q)) : 0.0;
        cand.push_back({j * G.nx + i, f, A});
      }
  }
  std::sort(cand.begin(), cand.end(), [](const Cand& a, const Cand& b) {
    if (a.cell != b.cell) return a.cell < b.cell;
    if (a.area != b.area) return a.area > b.area;
    return a.f < b.f;
  });

  const size_t base = cells.size();
  cells.resize(base + (size_t)ncell);
  size_t k = 0;
  for (int64_t cell = 0; cell < ncell; ++cell) {
    const size_t kb = k;
    while (k < cand.size() && cand[k].cell == cell) ++k;
    const int64_t i = cell % G.nx, j = cell / G.nx;
    const double x0 = G.ox + i * sx, x1 = x0 + sx, y0 = G.oy + j * sy, y1 = y0 + sy;
    const double Acell = sx * sy;
    CellRec& R = cells[base + (size_t)cell];
    R.a0 = R.b0 = R.a1 = R.b1 = 0.0;
    R.c0 = R.c1 = 1.0;
    // candidate list (fallback), ordered by overlap area
    const int32_t list_start = (int32_t)items.size();
    for (size_t q = kb; q < k; ++q) items.push_back(cand[q].f);
    const int32_t list_count = (int32_t)(k - kb);
    lists.push_back(list_start);
    lists.push_back(list_count);
    auto fallback = [&]() {
      R.a0 = R.b0 = R.a1 = R.b1 = 0.0;
      R.c0 = R.c1 = 1.0;
      R.leaf[0] = R.leaf[1] = R.leaf[2] = R.leaf[3] = -2;
      G.n_fallback++;
    };
    std::vector<int32_t> live;
    for (size_t q = kb; q < k; ++q)
      if (cand[q].area > 1e-12 * Acell) live.push_back(cand[q].f);
    if (live.empty()) {
      R.leaf[0] = R.leaf[1] = R.leaf[2] = R.leaf[3] = -1;
      G.n_outside++;
      continue;
    }
    bool ok = true;
    for (int32_t f : live) ok = ok && convex[f];
    if (!ok) {
      fallback();
      continue;
    }
    // distinct lines of candidate edges that cross the cell interior
    std::vector<Line> lines;
    const P2 corner[4] = {{x0, y0}, {x1, y0}, {x1, y1}, {x0, y1}};
    const double tol = 1e-9 * std::max(sx, sy);
    for (int32_t f : live) {
      const double* v = xy + 8 * (size_t)(first + f);
      int n = nv[first + f];
      for (int e = 0; e < n; ++e) {
        int e2 = (e + 1) % n;
        P2 p{v[2 * e], v[2 * e + 1]}, q{v[2 * e2], v[2 * e2 + 1]};
        if (seg_len_in_rect(p, q, x0, x1, y0, y1) <= tol) continue;
        Line L = hps[f][e];
        bool neg = false, pos = false;
        for (const P2& c : corner) {
          double s = L.a * c.x + L.b * c.y + L.c;
          neg |= s < -tol;
          pos |= s > tol;
        }
        if (!(neg && pos)) continue;
        if (L.a < 0 || (L.a == 0 && L.b < 0)) L = {-L.a, -L.b, -L.c};
        bool dup = false;
        for (const Line& M : lines)
          if (std::fabs(M.a - L.a) < 1e-12 && std::fabs(M.b - L.b) < 1e-12 &&
              std::fabs(M.c - L.c) < 1e-12 * (1.0 + std::fabs(L.c)))
            dup = true;
        if (!dup) lines.push_back(L);
      }
    }
    if (lines.size() > 2) {
      fallback();
      continue;
    }
    if (lines.size() >= 1) { R.a0 = lines[0].a; R.b0 = lines[0].b; R.c0 = lines[0].c; }
    if (lines.size() >= 2) { R.a1 = lines[1].a; R.b1 = lines[1].b; R.c1 = lines[1].c; }
    // classify every region (code = bit0: s0 < 0, bit1: s1 < 0)
    for (int code = 0; code < 4 && ok; ++code) {
      R.leaf[code] = -2;
      if ((code & 1) && lines.size() < 1) continue;
      if ((code & 2) && lines.size() < 2) continue;
      Poly reg = rect(x0, x1, y0, y1);
      for (size_t l = 0; l < lines.size(); ++l) {
        const Line& L = lines[l];
        reg = ((code >> l) & 1) ? clip_half(reg, -L.a, -L.b, -L.c) : clip_half(reg, L.a, L.b, L.c);
      }
      double Ar = reg.size() >= 3 ? std::fabs(area(reg)) : 0.0;
      if (Ar <= 1e-12 * Acell) continue;  // empty region: only rounding can land here -> list
      double inside_sum = 0.0;
      int owner = -1;
      for (int32_t f : live) {
        Poly in = clip_convex(reg, hps[f]);
        double Ain = in.size() >= 3 ? std::fabs(area(in)) : 0.0;
        inside_sum += Ain;
        if (Ain >= (1.0 - 1e-9) * Ar) owner = f;
      }
      if (owner >= 0) R.leaf[code] = owner;
      else if (inside_sum <= 1e-9 * Ar) R.leaf[code] = -1;
      else ok = false;
    }
    if (!ok) {
      fallback();
      continue;
    }
    G.n_bsp++;
  }
  return G;
}

}  // namespace rthx

// ---------------------------------------------------------------------------
// Host twin of the device lookup (rthx_device.h locate) for tests: builds one
// grid over `count` polygons and locates n points.  Exported for
// tests/test_grid.py only; not part of include/rthx.h.
// ---------------------------------------------------------------------------
using rthx::CellRec;
using rthx::GridBuild;
using rthx::build_cell_grid;

namespace {
bool pip(double px, double py, const double* xy, int n) {  // findFace2D.jl:77-101
  bool inside = false;
  int j = n - 1;
  for (int i = 0; i < n; ++i) {
    double xi = xy[2 * i], yi = xy[2 * i + 1], xj = xy[2 * j], yj = xy[2 * j + 1];
    if ((yi > py) != (yj > py)) {
      double ix = xi + (xj - xi) / (yj - yi) * (py - yi);
      if (px < ix) inside = !inside;
    }
    j = i;
  }
  return inside;
}
}  // namespace

extern "C" __attribute__((visibility("default"))) int rthx_debug_grid_locate(const int32_t* nv, const double* xy,
                                                                            int32_t count, const double* pts, int64_t n,
                                                                            int32_t* out, int64_t* stats) {
  std::vector<CellRec> cells;
  std::vector<int32_t> lists, items;
  GridBuild g = build_cell_grid(nv, xy, 0, count, 2.0, cells, lists, items);
  for (int64_t k = 0; k < n; ++k) {
    double px = pts[2 * k], py = pts[2 * k + 1];
    double fi = std::floor((px - g.ox) * g.inv_x), fj = std::floor((py - g.oy) * g.inv_y);
    int res = -1;
    bool done = false;
    if (fi >= 0 && fi < g.nx && fj >= 0 && fj < g.ny) {
      int cell = (int)fj * g.nx + (int)fi;
      const CellRec& c = cells[cell];
      double s0 = c.a0 * px + c.b0 * py + c.c0, s1 = c.a1 * px + c.b1 * py + c.c1;
      int leaf = c.leaf[(s0 < 0 ? 1 : 0) | (s1 < 0 ? 2 : 0)];
      if (leaf >= 0) { res = leaf; done = true; }
      else if (leaf == -2) {
        for (int q = lists[2 * cell]; q < lists[2 * cell] + lists[2 * cell + 1] && !done; ++q)
          if (pip(px, py, xy + 8 * (size_t)items[q], nv[items[q]])) { res = items[q]; done = true; }
      }
    }
    if (!done)
      for (int f = 0; f < count && !done; ++f)
        if (pip(px, py, xy + 8 * (size_t)f, nv[f])) { res = f; done = true; }
    out[k] = res;
  }
  if (stats) {
    stats[0] = g.nx; stats[1] = g.ny; stats[2] = g.n_bsp; stats[3] = g.n_fallback; stats[4] = g.n_outside;
  }
  return 0;
}
