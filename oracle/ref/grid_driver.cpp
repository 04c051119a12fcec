// oracle/ref/grid_driver.cpp — TEST INFRASTRUCTURE ONLY (the checker).
//
// C entry points around the reference's own, unmodified
// src/gridStructure.cpp and src/LineIterator.cpp, compiled in place from
// /root/reference by oracle/ref/Makefile into oracle/_ref/libref_grid.so.
// Both translation units include only the standard library
// (include/gridStructure.h, include/LineIterator.h), so no stand-in header is
// involved.  tests/test_ref_grid.py compares the oracle's restatements
// (oracle_line_coords, oracle_grid_candidates) with these.
#include <list>
#include <unordered_set>
#include <utility>

#include "gridStructure.h"
#include "LineIterator.h"

using namespace ORB_SLAM3;

// getLineCoords (gridStructure.cpp:32-40) -> (x, y) pairs in list order
extern "C" int ref_line_coords(double x1, double y1, double x2, double y2, int* out_xy, int cap) {
    std::list<std::pair<int, int>> l;
    getLineCoords(x1, y1, x2, y2, l);
    int n = 0;
    for (auto& p : l) {
        if (n < cap) { out_xy[2 * n] = p.first; out_xy[2 * n + 1] = p.second; }
        ++n;
    }
    return n;
}

// A GridStructure(rows, cols) filled with at(x, y).push_back in CSR order
// (cells x * rows + y), then get(sp) and get(ep) into one unordered_set as
// LineMatcher::matchGrid does (LineMatcher.cpp:226-227); the set's iteration
// order is written to out.  With this host's libstdc++ (GCC 11) the range
// insert passes no rehash hint: the oracle's range_hint = 0 mode.
extern "C" int ref_grid_candidates(int cols, int rows, const int* cell_off, const int* cell_idx, int spx, int spy,
                                   int epx, int epy, int w0, int w1, int h0, int h1, int* out, int cap) {
    GridStructure grid(rows, cols);
    for (int x = 0; x < cols; ++x)
        for (int y = 0; y < rows; ++y)
            for (int k = cell_off[x * rows + y]; k < cell_off[x * rows + y + 1]; ++k) grid.at(x, y).push_back(cell_idx[k]);
    GridWindow w;
    w.width = std::make_pair(w0, w1);
    w.height = std::make_pair(h0, h1);
    std::unordered_set<int> c;
    grid.get(spx, spy, w, c);
    grid.get(epx, epy, w, c);
    int n = 0;
    for (int v : c) {
        if (n < cap) out[n] = v;
        ++n;
    }
    return n;
}

// GridStructure::at out of range returns the shared out_of_bounds list
// (gridStructure.cpp:58-65): 1 if (x, y) is a grid cell
extern "C" int ref_grid_at_in_bounds(int cols, int rows, int x, int y) {
    GridStructure grid(rows, cols);
    std::list<int>& a = grid.at(x, y);
    std::list<int>& oob = grid.at(-1, -1);
    return &a != &oob;
}
