// siddhi-hip: the instantiations of k_sw_lean (the headline shape's solve) and
// k_sw_spill (spilled owners), and the dispatcher of k_sw_solve's units (sweep_solve.hip), in a
// unit of their own so the library's units build in parallel.
#include "sweep.h"

namespace shp {

#ifdef SW_LEAN_AGG  // the SHP_LAYOUT_AGG instantiations, a unit of their own (build.py)
void sw_launch_lean_agg(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                        const MatchOut& O, int* err) {
#define SA_CASE(c, p) \
  case c * 8 + p:                                                                                        \
    if (D.r12) {                                                                                         \
      if (B.seq) k_sw_lean<c, p, true, true, SwRec12><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);        \
      else k_sw_lean<c, p, true, false, SwRec12><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);             \
    } else {                                                                                             \
      if (B.seq) k_sw_lean<c, p, true, true, SwRec><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);          \
      else k_sw_lean<c, p, true, false, SwRec><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);               \
    }                                                                                                    \
    break;
  switch (ct * 8 + opc) {
    SA_CASE(1, 1) SA_CASE(1, 2) SA_CASE(1, 3) SA_CASE(1, 4) SA_CASE(1, 5) SA_CASE(1, 6)
    SA_CASE(2, 1) SA_CASE(2, 2) SA_CASE(2, 3) SA_CASE(2, 4) SA_CASE(2, 5) SA_CASE(2, 6)
    default: break;
  }
#undef SA_CASE
}
#else

void sw_launch_solve_nt1_0(int, int, unsigned, hipStream_t, const SweepDev&, const BatchView&, const MatchOut&, int*);
void sw_launch_solve_nt1_1(int, int, unsigned, hipStream_t, const SweepDev&, const BatchView&, const MatchOut&, int*);
void sw_launch_solve_nt1_2(int, int, unsigned, hipStream_t, const SweepDev&, const BatchView&, const MatchOut&, int*);

void sw_launch_solve(int nt1, int nt2, int ct, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                     const MatchOut& O, int* err) {
  if (nt1 == 0) sw_launch_solve_nt1_0(nt2, ct, grid, s, D, B, O, err);
  else if (nt1 == 1) sw_launch_solve_nt1_1(nt2, ct, grid, s, D, B, O, err);
  else if (nt1 == 2) sw_launch_solve_nt1_2(nt2, ct, grid, s, D, B, O, err);
}

void sw_launch_lean(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                    const MatchOut& O, int* err) {
#define SL_CASE(c, p) \
  case c * 8 + p:                                                                                        \
    if (D.r12) {                                                                                         \
      if (B.seq) k_sw_lean<c, p, false, true, SwRec12><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);       \
      else k_sw_lean<c, p, false, false, SwRec12><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);            \
    } else {                                                                                             \
      if (B.seq) k_sw_lean<c, p, false, true, SwRec><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);         \
      else k_sw_lean<c, p, false, false, SwRec><<<grid, SL_THREADS, 0, s>>>(D, B, O, err);              \
    }                                                                                                    \
    break;
  switch (ct * 8 + opc) {
    SL_CASE(1, 1) SL_CASE(1, 2) SL_CASE(1, 3) SL_CASE(1, 4) SL_CASE(1, 5) SL_CASE(1, 6)
    SL_CASE(2, 1) SL_CASE(2, 2) SL_CASE(2, 3) SL_CASE(2, 4) SL_CASE(2, 5) SL_CASE(2, 6)
    default: break;
  }
#undef SL_CASE
}

// k_sw_win (sweep_win.h): one 64-lane wave per unit of SWW_U records, then one per owner
void sw_launch_win(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                   const MatchOut& O, int* err) {
#define SW_CASE(c, p) \
  case c * 8 + p: k_sw_win<c, p><<<grid, 64, 0, s>>>(D, B, O, err); break;
  switch (ct * 8 + opc) {
    SW_CASE(1, 1) SW_CASE(1, 2) SW_CASE(1, 3) SW_CASE(1, 4) SW_CASE(1, 5) SW_CASE(1, 6)
    SW_CASE(2, 1) SW_CASE(2, 2) SW_CASE(2, 3) SW_CASE(2, 4) SW_CASE(2, 5) SW_CASE(2, 6)
    default: break;
  }
#undef SW_CASE
}

void sw_launch_win_tail(int ct, int opc, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                        int* err) {
#define SW_CASE(c, p) \
  case c * 8 + p: k_sw_win_tail<c, p><<<grid, 64, 0, s>>>(D, B, err); break;
  switch (ct * 8 + opc) {
    SW_CASE(1, 1) SW_CASE(1, 2) SW_CASE(1, 3) SW_CASE(1, 4) SW_CASE(1, 5) SW_CASE(1, 6)
    SW_CASE(2, 1) SW_CASE(2, 2) SW_CASE(2, 3) SW_CASE(2, 4) SW_CASE(2, 5) SW_CASE(2, 6)
    default: break;
  }
#undef SW_CASE
}

void sw_launch_spill(int nt2, int ct, unsigned grid, hipStream_t s, const SweepDev& D, const BatchView& B,
                     const MatchOut& O, int* err) {
  switch (nt2 * 3 + ct) {
#define SP_CASE(b, c) \
  case b * 3 + c: k_sw_spill<b, c><<<grid, SP_THREADS, 0, s>>>(D, B, O, err); break;
    SP_CASE(0, 0) SP_CASE(0, 1) SP_CASE(0, 2) SP_CASE(1, 0) SP_CASE(1, 1) SP_CASE(1, 2)
    SP_CASE(2, 0) SP_CASE(2, 1) SP_CASE(2, 2)
#undef SP_CASE
    default: break;
  }
}

#endif  // SW_LEAN_AGG

}  // namespace shp
