// rthx_grid.h — host-side builder of the device point-location grid
// (DESIGN.md "Point location").
#pragma once

#include <stdint.h>

#include <vector>

namespace rthx {

// One cell of the device grid: a two-line decision record.  A point p of
// the cell has code  (s0(p) < 0) | (s1(p) < 0) << 1  with  s = a x + b y + c
// for lines 0 and 1 (an absent line is a = b = 0, c = 1, i.e. always >= 0),
// and lies in polygon leaf[code]:
//   leaf >= 0  polygon index (local to the set)
//   leaf == -1 outside every polygon of the set (the reference's grid test
//              fails; the bbox scan decides)
//   leaf == -2 fallback: test the cell's candidates (lists[2*cell] = start,
//              lists[2*cell+1] = count into items, ordered by overlap area)
//              in order with the point-in-polygon test.
struct alignas(16) CellRec {
  double a0, b0, c0;
  double a1, b1, c1;
  int32_t leaf[4];
};
static_assert(sizeof(CellRec) == 64, "CellRec must be 64 bytes");

struct GridBuild {
  double ox, oy, inv_x, inv_y;
  int32_t nx, ny;
  int64_t n_bsp = 0, n_fallback = 0, n_outside = 0;  // statistics
};

// Build the grid over polygons [first, first+count) (vertices xy[8*i..],
// nv[i] in {3,4}), appending one record per cell to `cells`, one (start,
// count) pair per cell to `lists` and the candidate lists to `items`.  `cells_per_extent` sets the cell size relative to the mean
// polygon bbox extent per axis.
GridBuild build_cell_grid(const int32_t* nv, const double* xy, int first, int count, double cells_per_extent,
                          std::vector<CellRec>& cells, std::vector<int32_t>& lists, std::vector<int32_t>& items);

}  // namespace rthx
