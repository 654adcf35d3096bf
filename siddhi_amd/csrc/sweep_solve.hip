// siddhi-hip: k_sw_solve's instantiations for one e1 filter term count (SW_NT1 = 0, 1, 2: build.py
// compiles this file once per value), the library's largest kernel family split across units
// so they build in parallel.  sweep_lean.hip holds the dispatcher sw_launch_solve.
#include "sweep.h"

#ifndef SW_NT1
#error "sweep_solve.hip is built with -DSW_NT1=0|1|2"
#endif

namespace shp {

#define SW_FN_(n) sw_launch_solve_nt1_##n
#define SW_FN(n) SW_FN_(n)
void SW_FN(SW_NT1)(int nt2, int ct, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                   const MatchOut& O, int* err) {
  switch (nt2 * 3 + ct) {
#define SW_CASE(b, c) \
  case b * 3 + c: k_sw_solve<SW_NT1, b, c><<<grid, SWS_THREADS, 0, s>>>(D, B, O, err); break;
    SW_CASE(0, 0) SW_CASE(0, 1) SW_CASE(0, 2) SW_CASE(1, 0) SW_CASE(1, 1) SW_CASE(1, 2)
    SW_CASE(2, 0) SW_CASE(2, 1) SW_CASE(2, 2)
#undef SW_CASE
    default: break;
  }
}

}  // namespace shp
