// psg_kernels.hpp — launcher declarations (one translation unit per algorithm).
#pragma once
#ifndef __HIPCC_RTC__  // (a hiprtc build of a fused Spec module has no host launchers)
#include <hip/hip_runtime.h>

namespace psg {
struct KArgs;
struct VmArgs;
struct PopArgs;

hipError_t launch_otr(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_lv(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_floodmin(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_kset(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_benor(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_otr2(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_slv(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_kset_es(const KArgs& a, int W, int grid, hipStream_t s);
hipError_t launch_epsilon(const KArgs& a, int W, int grid, hipStream_t s);

const void* otr_kernel_ptr(int W);
const void* lv_kernel_ptr(int W);
const void* floodmin_kernel_ptr(int W);
const void* kset_kernel_ptr(int W);
const void* benor_kernel_ptr(int W);
const void* otr2_kernel_ptr(int W);
const void* slv_kernel_ptr(int W);
const void* kset_es_kernel_ptr(int W);
const void* epsilon_kernel_ptr(int W);

hipError_t launch_champ_selftest(const uint64_t* sets, int count, int tiebreak, int32_t* out, hipStream_t s);
hipError_t launch_schedule(const KArgs& a, int W, int grid, uint64_t* ho_out, int32_t* crash_out, hipStream_t s);
hipError_t launch_population(const PopArgs& a, hipStream_t s);
hipError_t launch_spec_vm(const VmArgs& a, int grid, hipStream_t s);
hipError_t launch_gen_init(uint64_t inst_begin, uint64_t count, int n, int alg, int V, uint64_t seed, int32_t* out,
                           hipStream_t s);
}  // namespace psg
#endif
