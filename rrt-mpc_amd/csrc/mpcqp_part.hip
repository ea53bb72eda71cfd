// mpcqp_part.hip -- explicit instantiations of the solver (and of the fused fleet loop) for horizons
// [MPCQP_PART_LO, MPCQP_PART_HI] (the library is built from several such objects in parallel).
#include "mpcqp_solve.h"

#if !defined(MPCQP_PART_LO) || !defined(MPCQP_PART_HI)
#error "define MPCQP_PART_LO and MPCQP_PART_HI"
#endif

#ifdef MPCQP_STAMPS
// diagnostic builds: this object's own g_stamps (every translation unit has its copy) joins the
// registry mpcqp_debug_stamps sums over
extern "C" void mpcqp_register_stamps(hipError_t (*f)(unsigned long long*, int));
namespace {
hipError_t part_stamps(unsigned long long* out32, int reset) {
  hipError_t e = hipSuccess;
  if (out32) {
    unsigned long long v[32];
    e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_stamps), sizeof(v));
    for (int i = 0; i < 32 && e == hipSuccess; ++i) out32[i] += v[i];
  }
  if (e == hipSuccess && reset) {
    unsigned long long z[32] = {0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z));
  }
  return e;
}
const int kRegistered = (mpcqp_register_stamps(part_stamps), 0);
}  // namespace
#endif

namespace mpcqp {
#if MPCQP_PART_LO <= 1 && 1 <= MPCQP_PART_HI
template void launch_solve<1>(hipStream_t, const Launch&);
template bool launch_solve_pair<1>(hipStream_t, const Launch&);
template void launch_serve<1>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<1>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 2 && 2 <= MPCQP_PART_HI
template void launch_solve<2>(hipStream_t, const Launch&);
template bool launch_solve_pair<2>(hipStream_t, const Launch&);
template void launch_serve<2>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<2>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 3 && 3 <= MPCQP_PART_HI
template void launch_solve<3>(hipStream_t, const Launch&);
template bool launch_solve_pair<3>(hipStream_t, const Launch&);
template void launch_serve<3>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<3>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 4 && 4 <= MPCQP_PART_HI
template void launch_solve<4>(hipStream_t, const Launch&);
template bool launch_solve_pair<4>(hipStream_t, const Launch&);
template void launch_serve<4>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<4>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 5 && 5 <= MPCQP_PART_HI
template void launch_solve<5>(hipStream_t, const Launch&);
template bool launch_solve_pair<5>(hipStream_t, const Launch&);
template void launch_serve<5>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<5>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 6 && 6 <= MPCQP_PART_HI
template void launch_solve<6>(hipStream_t, const Launch&);
template bool launch_solve_pair<6>(hipStream_t, const Launch&);
template void launch_serve<6>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<6>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 7 && 7 <= MPCQP_PART_HI
template void launch_solve<7>(hipStream_t, const Launch&);
template bool launch_solve_pair<7>(hipStream_t, const Launch&);
template void launch_serve<7>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<7>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 8 && 8 <= MPCQP_PART_HI
template void launch_solve<8>(hipStream_t, const Launch&);
template bool launch_solve_pair<8>(hipStream_t, const Launch&);
template void launch_serve<8>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<8>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 9 && 9 <= MPCQP_PART_HI
template void launch_solve<9>(hipStream_t, const Launch&);
template bool launch_solve_pair<9>(hipStream_t, const Launch&);
template void launch_serve<9>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<9>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 10 && 10 <= MPCQP_PART_HI
template void launch_solve<10>(hipStream_t, const Launch&);
template bool launch_solve_pair<10>(hipStream_t, const Launch&);
template void launch_serve<10>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<10>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 11 && 11 <= MPCQP_PART_HI
template void launch_solve<11>(hipStream_t, const Launch&);
template bool launch_solve_pair<11>(hipStream_t, const Launch&);
template void launch_serve<11>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<11>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 12 && 12 <= MPCQP_PART_HI
template void launch_solve<12>(hipStream_t, const Launch&);
template bool launch_solve_pair<12>(hipStream_t, const Launch&);
template void launch_serve<12>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<12>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 13 && 13 <= MPCQP_PART_HI
template void launch_solve<13>(hipStream_t, const Launch&);
template bool launch_solve_pair<13>(hipStream_t, const Launch&);
template void launch_serve<13>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<13>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 14 && 14 <= MPCQP_PART_HI
template void launch_solve<14>(hipStream_t, const Launch&);
template bool launch_solve_pair<14>(hipStream_t, const Launch&);
template void launch_serve<14>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<14>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 15 && 15 <= MPCQP_PART_HI
template void launch_solve<15>(hipStream_t, const Launch&);
template bool launch_solve_pair<15>(hipStream_t, const Launch&);
template void launch_serve<15>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<15>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 16 && 16 <= MPCQP_PART_HI
template void launch_solve<16>(hipStream_t, const Launch&);
template void launch_serve<16>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<16>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 17 && 17 <= MPCQP_PART_HI
template void launch_solve<17>(hipStream_t, const Launch&);
template void launch_serve<17>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<17>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 18 && 18 <= MPCQP_PART_HI
template void launch_solve<18>(hipStream_t, const Launch&);
template void launch_serve<18>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<18>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 19 && 19 <= MPCQP_PART_HI
template void launch_solve<19>(hipStream_t, const Launch&);
template void launch_serve<19>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<19>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 20 && 20 <= MPCQP_PART_HI
template void launch_solve<20>(hipStream_t, const Launch&);
template void launch_serve<20>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<20>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 21 && 21 <= MPCQP_PART_HI
template void launch_solve<21>(hipStream_t, const Launch&);
template void launch_serve<21>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<21>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 22 && 22 <= MPCQP_PART_HI
template void launch_solve<22>(hipStream_t, const Launch&);
template void launch_serve<22>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<22>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 23 && 23 <= MPCQP_PART_HI
template void launch_solve<23>(hipStream_t, const Launch&);
template void launch_serve<23>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<23>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 24 && 24 <= MPCQP_PART_HI
template void launch_solve<24>(hipStream_t, const Launch&);
template void launch_serve<24>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<24>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 25 && 25 <= MPCQP_PART_HI
template void launch_solve<25>(hipStream_t, const Launch&);
template void launch_serve<25>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<25>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 26 && 26 <= MPCQP_PART_HI
template void launch_solve<26>(hipStream_t, const Launch&);
template void launch_serve<26>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<26>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 27 && 27 <= MPCQP_PART_HI
template void launch_solve<27>(hipStream_t, const Launch&);
template void launch_serve<27>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<27>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 28 && 28 <= MPCQP_PART_HI
template void launch_solve<28>(hipStream_t, const Launch&);
template void launch_serve<28>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<28>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 29 && 29 <= MPCQP_PART_HI
template void launch_solve<29>(hipStream_t, const Launch&);
template void launch_serve<29>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<29>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 30 && 30 <= MPCQP_PART_HI
template void launch_solve<30>(hipStream_t, const Launch&);
template void launch_serve<30>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<30>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 31 && 31 <= MPCQP_PART_HI
template void launch_solve<31>(hipStream_t, const Launch&);
template void launch_serve<31>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<31>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
#if MPCQP_PART_LO <= 32 && 32 <= MPCQP_PART_HI
template void launch_solve<32>(hipStream_t, const Launch&);
template void launch_serve<32>(hipStream_t, const mpcqp_params&, const ServeLaunch&);
template void launch_fleet_loop<32>(hipStream_t, const mpcqp_params*, const mpcqp_fleet&, int,
                                           const LoopTrigger&);
#endif
}  // namespace mpcqp
