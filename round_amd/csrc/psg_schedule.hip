// psg_schedule.hip — export of the seeded HO schedule (psg_materialize_schedule).
//
// The round kernels draw HO(p, k) on the fly (Sched<W>::ho, never stored). This
// kernel runs the same generator and writes the sets to HBM in the explicit
// schedule layout ho[inst][k][p][W] plus the crash rounds crash[inst][p], so
// that a caller (the in-JVM harness of SURVEY §8c, the adversary search,
// counterexample files) can replay an instance with psg_load_schedule, or
// drive the reference's own Round.send/update with the very same HO sets.
// The HO sets of a round do not depend on process state (faults are HO sets,
// psync/Process.scala:14), so every round is exported, including rounds after
// all processes halted.
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

template <int W>
__global__ void __launch_bounds__(Geometry<W>::kThreads) schedule_kernel(KArgs a, uint64_t* ho_out, int32_t* crash_out) {
  __shared__ uint64_t xb[Grp<W>::kXb];
  __shared__ int64_t red[2 * W];
  Grp<W> g;
  grp_setup(g, a, xb, red);
  constexpr int G = Geometry<W>::kGroups;
  const int grp = W == 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int n = a.n;
  for (uint64_t i = (uint64_t)blockIdx.x * G + grp; i < a.count; i += (uint64_t)gridDim.x * G) {
    const uint64_t inst = a.inst_begin + i;
    Sched<W> sc;
    sc.setup(a, inst, g.pid, g.valid);
    sc.prep_good(0, g.lane, a.R);
    if (crash_out && g.valid) crash_out[i * (uint64_t)n + g.pid] = sc.crash_round;
    for (int k = 0; k < a.R; ++k) {
      Mask<W> goodS;
      const bool good = sc.good_round(k, g.lane, a.R, goodS);
      Mask<W> CB = mzero<W>(), CN = mzero<W>();
      if (sc.crash_on) {
        CB = g.ballot(sc.crash_round >= 0 && sc.crash_round < k);
        CN = g.ballot(sc.crash_round == k);
      }
      const Mask<W> HO = sc.ho(k, g.pid, good, goodS, CB, CN);
      if (g.valid) {
        uint64_t* q = ho_out + ((i * (uint64_t)a.R + (uint64_t)k) * (uint64_t)n + (uint64_t)g.pid) * W;
#pragma unroll
        for (int w = 0; w < W; ++w) q[w] = HO.w[w];
      }
    }
  }
}

hipError_t launch_schedule(const KArgs& a, int W, int grid, uint64_t* ho_out, int32_t* crash_out, hipStream_t s) {
  switch (W) {
    case 1: hipLaunchKernelGGL(schedule_kernel<1>, dim3(grid), dim3(Geometry<1>::kThreads), 0, s, a, ho_out, crash_out); break;
    case 2: hipLaunchKernelGGL(schedule_kernel<2>, dim3(grid), dim3(Geometry<2>::kThreads), 0, s, a, ho_out, crash_out); break;
    case 3: hipLaunchKernelGGL(schedule_kernel<3>, dim3(grid), dim3(Geometry<3>::kThreads), 0, s, a, ho_out, crash_out); break;
    case 4: hipLaunchKernelGGL(schedule_kernel<4>, dim3(grid), dim3(Geometry<4>::kThreads), 0, s, a, ho_out, crash_out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace psg
