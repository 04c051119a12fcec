// oracle/ref_fma.h — TEST INFRASTRUCTURE ONLY.
//
// The multiply-adds the reference build fuses.  The reference's own sources
// are compiled by GCC 9.4 with `-O3 -march=native` (CMakeLists.txt; the
// shipped build/CMakeFiles/ORB_SLAM3-Relocalization.dir/flags.make), and
// GCC's C++ front end contracts `a*b + c` into one fused multiply-add even
// under -std=c++11 (only its C front end turns contraction off for ISO
// modes).  The shipped objects (build/CMakeFiles/.../src/*.o) show which
// expressions were fused; tests/test_ref_objects.py pins every site on the
// path by disassembling them (never executed).  The oracle is built
// -ffp-contract=off, so the calls below are its only fused operations.  For
// `a*b + c*d` GCC fuses the left product: ref_fma(a, b, c*d).
//
// The third-party line_descriptor library (LSDDetector_custom.cpp,
// binary_descriptor_custom.cpp) is built `-O3 -mtune=native` without
// -march: plain SSE2, no fused operation anywhere (also pinned).
//
// -DORACLE_NO_REF_FMA builds the unfused variant (tools/fma_impact.py
// measures how many outputs the contraction changes).
#pragma once
#include <cmath>

#ifdef ORACLE_NO_REF_FMA
static inline double ref_fma(double a, double b, double c) { return a * b + c; }
static inline float ref_fmaf(float a, float b, float c) { return a * b + c; }
#else
static inline double ref_fma(double a, double b, double c) { return std::fma(a, b, c); }
static inline float ref_fmaf(float a, float b, float c) { return std::fma(a, b, c); }
#endif
