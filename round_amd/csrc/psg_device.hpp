// psg_device.hpp — device building blocks for the MI355X (gfx950) HO executor.
//
// Execution model: one wave64 executes one instance, one lane per process
// (pid = lane) for n <= 64; for n > 64 a workgroup of W = ceil(n/64) waves
// executes one instance and cross-wave primitives exchange 64-bit ballot words
// through LDS. HO sets are W x 64-bit masks generated on the device from a
// counter-based RNG and never touch HBM. Mailbox primitives are ballots,
// popcounts and shuffles over those masks.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <stdint.h>
#else  // hiprtc (psg_spec_compile_native): the runtime is implicit, its integer types are namespaced
using __hip_internal::int8_t;
using __hip_internal::int16_t;
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#define INT32_MIN (-2147483647 - 1)
#define INT32_MAX 2147483647
#define INT64_MIN (-9223372036854775807LL - 1)
#define INT64_MAX 9223372036854775807LL
#endif

#include "../../include/psg.h"

#define PSG_DEV __device__ __forceinline__

namespace psg {

// A compile-time phase slot passed to a generic lambda (the round loops specialise each slot's
// step): a tag of our own, since hiprtc (psg_spec_compile_native) has no <type_traits>
template <int K>
struct Slot {
  static constexpr int value = K;
};

// ---------------------------------------------------------------- kernel args
struct KArgs {
  uint64_t inst_begin;
  uint64_t count;
  const uint64_t* ids;               // nullable: explicit global instance ids
  const int32_t* init;               // nullable: [count][n] initial values (else seeded)
  int32_t* out_decision;             // nullable: [count][n]
  uint8_t* out_dround;               // nullable: [count][n], 0xFF = none
  psg_instance_summary* out_inst;    // nullable: [count]
  psg_process_record* out_rec;       // nullable: [count][n]
  unsigned long long* counters;      // [NCOUNTERS]
  uint64_t seed;
  const double* init_f64;            // nullable: [count][n] Double initial values (EpsilonConsensus)
  double* out_dec_f64;               // nullable: [count][n] Double decisions
  double* out_rec_f64;               // nullable: [count][n][2] (decision, final x) for the fetch path
  double real_param;                 // EpsilonConsensus epsilon
  int32_t* trace;                    // nullable: Spec-program trace [count][R+1][PSG_NFIELDS][n]
  uint32_t trace_fields;             // bit f: field f is traced (the fields the Spec program reads)
  int32_t n, R, V, param, param2, variant, tiebreak;
  uint32_t drop_log2, good_p32;
  int32_t good_min, crash_fmax, ho_min;
  uint32_t self_bit;
  // explicit schedule (psg_load_schedule): HO(p, k) of global instance id `inst` is
  // ho_in[((inst - ho_base) * R + k) * n + p][0..W-1]; crash_in[(inst - ho_base) * n + p]
  // (nullable) = crash round for the never-crashed classification, -1 = correct
  const uint64_t* ho_in;
  const int32_t* crash_in;
  uint64_t ho_base;
  uint64_t init_base;  // fetch path with staged inputs: init row of id `inst` is inst - init_base
  // packed KSet's hand-off from the general-round kernel to the uniform-t tail kernel
  // (psg_kset.hip): per batch row a header word, 64 per-lane state words and the decisions of
  // the processes halted before the hand-off ([row][n])
  uint64_t* hand_hdr;
  uint64_t* hand_meta;
  int32_t* hand_dec;
};

// Initial value of process pid of batch element i (global id inst): staged rows
// are indexed by batch position, or by global id in the fetch (ids) path.
PSG_DEV uint64_t init_row(const KArgs& a, uint64_t i, uint64_t inst) { return a.ids ? inst - a.init_base : i; }
// Host-supplied initial value of process pid (a.init non-null). The pid term of the address is
// formed here per instance (opaque copy), not hoisted out of the instance loop and kept live.
PSG_DEV int32_t init_x(const KArgs& a, uint64_t i, uint64_t inst, int pid) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(pid));
#endif
  return a.init[init_row(a, i, inst) * (uint64_t)a.n + (uint64_t)pid];
}

// Spec-program interpreter arguments (psg_spec_vm.hip)
struct VmArgs {
  const int32_t* code;
  const int32_t* slot_entry;
  const int32_t* slot_flags;
  int32_t n_slots, term_entry, n_words;
  const int32_t* trace;  // [count][R+1][PSG_NFIELDS][n]
  uint64_t count;
  int32_t n, R;
  psg_instance_summary* out_inst;
  unsigned long long* counters;  // NCOUNTERS (fail counts, termination histogram)
  int32_t* err;                  // OR of VM_ERR_* over all instances
};

// Search-population kernels (psg_population.hip)
struct PopArgs {
  uint64_t* ho;             // destination population [count][R][n][W]
  const uint64_t* src;      // current population (next generation), null for fresh
  int32_t* init;            // destination initial values [count][n]
  const int32_t* src_init;  // current initial values
  const uint32_t* parent;   // [count] (null for fresh)
  const uint8_t* op;        // [count] 0 copy, 1 mutate, 2 fresh (null: all fresh)
  uint64_t count;
  int n, R, W;
  uint64_t seed;
  uint32_t gen, flips;
  int32_t min_size;
  uint32_t self_bit;
  uint32_t keep[4];
  int32_t V;
  uint32_t redraw;
  int benor;
};

#ifndef PSG_PHASE_TIMERS
#define PSG_PHASE_TIMERS 0
#endif
// global counter layout (uint64 each)
enum { C_FAIL = 0, C_DECIDED = PSG_MAX_CHECKS, C_DIGEST = PSG_MAX_CHECKS + 1,
       C_ACTIVE = PSG_MAX_CHECKS + 2,  // process-rounds in which the process took a step
       C_LIVE = PSG_MAX_CHECKS + 3,    // instance-rounds with some process still active
       C_HIST = PSG_MAX_CHECKS + 4,
       NCOUNTERS = C_HIST + PSG_MAX_ROUNDS + 2,
       // profiling builds only (-DPSG_PHASE_TIMERS=1): per-phase shader cycles summed over waves
       // (4 phase slots, then wave-lifetime s_memrealtime ticks summed, ~min start, max end, waves)
       // (4 phase slots, then wave-lifetime s_memrealtime ticks summed, ~min start, max end, waves,
       // then (start, end) per wave for the first 16384 waves)
       // instance queues (InstanceQueue): NQUEUES counters, one per 128 B line
       // (two regions: a launch's second kernel — packed KSet's uniform-t tail — takes its own)
       C_QUEUE = NCOUNTERS, NQUEUES = 8, QUEUE_STRIDE = 16, NQUEUE_REGIONS = 2,
       C_TIMER = C_QUEUE + NQUEUE_REGIONS * NQUEUES * QUEUE_STRIDE, NTIMERS = 8, NSTAMP_WAVES = 16384,
       T_RT_SUM = NTIMERS, T_RT_MIN = NTIMERS + 1, T_RT_MAX = NTIMERS + 2, T_WAVES = NTIMERS + 3,
       T_STAMPS = NTIMERS + 4,
       NTIMER_SLOTS = PSG_PHASE_TIMERS ? T_STAMPS + 2 * NSTAMP_WAVES : 0, NCOUNTERS_ALLOC = C_TIMER + NTIMER_SLOTS };

// Phase timers of a profiling build: t.mark(j) charges the cycles since the last
// mark to phase j (uniform, kept in SGPRs); flush adds them to the global slots.
struct PhaseTimers {
#if PSG_PHASE_TIMERS
  uint64_t last, rt0, acc[NTIMERS];
  PSG_DEV void start() {
    for (int j = 0; j < NTIMERS; ++j) acc[j] = 0;
    rt0 = __builtin_amdgcn_s_memrealtime();
    last = __builtin_amdgcn_s_memtime();
  }
  PSG_DEV void mark(int j) {
#if PSG_PHASE_TIMERS == 1
    const uint64_t t = __builtin_amdgcn_s_memtime();
    acc[j] += t - last;
    last = t;
#endif
  }
  // event-count builds (-DPSG_PHASE_TIMERS=2): mark() is off, the slots count events instead
  PSG_DEV void add(int j, uint64_t v) {
#if PSG_PHASE_TIMERS == 2
    acc[j] += v;
#endif
  }
  PSG_DEV void flush(unsigned long long* g, int lane) {
    const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {
      for (int j = 0; j < NTIMERS; ++j) atomicAdd(&g[C_TIMER + j], (unsigned long long)acc[j]);
      atomicAdd(&g[C_TIMER + T_RT_SUM], (unsigned long long)(rt1 - rt0));
      atomicMax(&g[C_TIMER + T_RT_MIN], (unsigned long long)~rt0);
      atomicMax(&g[C_TIMER + T_RT_MAX], (unsigned long long)rt1);
      atomicAdd(&g[C_TIMER + T_WAVES], 1ull);
      const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
      if (wave < NSTAMP_WAVES) {
        g[C_TIMER + T_STAMPS + 2 * wave] = rt0;
        g[C_TIMER + T_STAMPS + 1 + 2 * wave] = rt1;
      }
    }
  }
#else
  PSG_DEV void start() {}
  PSG_DEV void mark(int) {}
  PSG_DEV void add(int, uint64_t) {}
  PSG_DEV void flush(unsigned long long*, int) {}
#endif
};

constexpr uint32_t ROUND_INIT = 0xFFFFFFFFu;
constexpr uint32_t ROUND_CRASH = 0xFFFFFFFEu;
constexpr uint32_t PID_GLOBAL = 0xFFFFu;
constexpr uint32_t COIN_TAG = 0x80000000u;

// ---------------------------------------------------------------- Philox4x32-10
struct U4 { uint32_t x, y, z, w; };

// a ^ b ^ c in one VALU instruction: gfx950 v_bitop3_b32 with truth table 0x96
// (hipcc otherwise emits two v_xor_b32 for the Philox mix)
PSG_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// Philox's 32x32 -> 64-bit products as one v_mad_u64_u32 each (the compiler's v_mul_lo_u32 +
// v_mul_hi_u32 pair measured 7 % slower per call, round-4 microbenchmark; the headline -1.4 %).
// Round 0's products stay in C: their operands are often wave-uniform (scalar multiplies).
#ifndef PSG_PHILOX_OPAQUE_KEYS
#define PSG_PHILOX_OPAQUE_KEYS 0
#endif
#ifndef PSG_PHILOX_MAD64
#define PSG_PHILOX_MAD64 2  // 2: carry-out in VCC (no SGPR pair per product: fused OTR -1.8 %, round-4 A/B)
#endif
#if PSG_PHILOX_MAD64 && defined(__HIP_DEVICE_COMPILE__)
PSG_DEV uint64_t mul64_mad(uint32_t a, uint32_t b) {
  uint64_t r;
#if PSG_PHILOX_MAD64 == 2  // carry-out into VCC (clobbered): no SGPR pair allocated per product
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b) : "vcc");
#else
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(r), "=s"(cy) : "v"(a), "v"(b));
#endif
  return r;
}
#define PSG_MUL64(r, a, b) ((r) == 0 ? (uint64_t)(a) * (b) : mul64_mad((a), (b)))
#else
#define PSG_MUL64(r, a, b) ((uint64_t)(a) * (b))
#endif
PSG_DEV U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#if PSG_PHILOX_OPAQUE_KEYS && defined(__HIP_DEVICE_COMPILE__)
  // the round keys are formed per call (18 scalar adds) instead of hoisted out of the kernel's
  // loops into 20 SGPRs that then spill to VGPR lanes
  asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = PSG_MUL64(r, 0xD2511F53u, c0);
    const uint64_t p1 = PSG_MUL64(r, 0xCD9E8D57u, c2);
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// 64-bit word j of a stream: call s = j/2 with ctr3 = base + (s << 16).
PSG_DEV uint64_t rword(uint64_t seed, uint64_t inst, uint32_t round, uint32_t ctr3base, uint32_t j) {
  U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), round, ctr3base + ((j >> 1) << 16), (uint32_t)seed,
                  (uint32_t)(seed >> 32));
  return (j & 1u) ? ((uint64_t)o.z | ((uint64_t)o.w << 32)) : ((uint64_t)o.x | ((uint64_t)o.y << 32));
}

// Sequential reader of a word stream, computing each Philox call once.
struct WordStream {
  uint64_t seed, inst;
  uint32_t round, base;
  int32_t cur;  // call index held in lo/hi, -1 = none
  uint64_t lo, hi;
  PSG_DEV WordStream(uint64_t s, uint64_t i, uint32_t r, uint32_t b) : seed(s), inst(i), round(r), base(b), cur(-1), lo(0), hi(0) {}
  PSG_DEV uint64_t word(uint32_t j) {
    const int32_t s = (int32_t)(j >> 1);
    if (s != cur) {
      U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), round, base + ((uint32_t)s << 16), (uint32_t)seed,
                      (uint32_t)(seed >> 32));
      lo = (uint64_t)o.x | ((uint64_t)o.y << 32);
      hi = (uint64_t)o.z | ((uint64_t)o.w << 32);
      cur = s;
    }
    return (j & 1u) ? hi : lo;
  }
};

PSG_DEV uint32_t mulhi32(uint32_t a, uint32_t b) { return __umulhi(a, b); }

// java.util.Random(s).nextBoolean(): BenOr coin (example/BenOr.scala:77)
PSG_DEV bool java_first_boolean(uint64_t s) {
  const uint64_t mult = 0x5DEECE66DULL, mask = (1ULL << 48) - 1;
  uint64_t seed = (s ^ mult) & mask;
  seed = (seed * mult + 0xBULL) & mask;
  return (seed >> 47) != 0;
}

// scala.collection.Hashing.improve on ProcessID.## (= id)
PSG_DEV uint32_t scala_improve(uint32_t h) {
  uint32_t x = h + ~(h << 9);
  x ^= (x >> 14);
  x += (x << 4);
  x ^= (x >> 10);
  return x;
}

// Sort key of an entry in a CHAMP trie given its payload depth (max shared
// 5-bit hash-prefix length with any other entry of the map): level by level
// from the root, (sub-node flag, fragment); payloads precede sub-nodes.
PSG_DEV uint64_t champ_key(uint32_t h, int depth) {
  uint64_t key = 0;
#pragma unroll
  for (int l = 0; l < 7; ++l) {
    const uint32_t frag = (h >> (5 * l)) & 31u;
    const uint64_t unit = l < depth ? (32u | frag) : (l == depth ? frag : 0u);
    key = (key << 6) | unit;
  }
  return key;
}

PSG_DEV int champ_cpl(uint32_t a, uint32_t b) {  // shared leading fragments, a != b
  int t = __builtin_ctz(a ^ b);
  return t / 5;
}


// ---------------------------------------------------------------- digest
PSG_DEV uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
template <bool OPAQUE = true>
PSG_DEV uint64_t proc_digest(int pid, int32_t dec, int32_t dround, int32_t hround, int32_t mainx) {
#if defined(__HIP_DEVICE_COMPILE__)
  // opaque copy: the pid term is recomputed per instance instead of hoisted out of the instance
  // loop and kept live (spilled to scratch) across every round (packed KSet's 12 B of scratch,
  // FloodMin -2..5 %); packed BenOr keeps the hoisted form (3.6 % faster, round-4 A/B)
  if constexpr (OPAQUE) asm volatile("" : "+v"(pid));
#endif
  uint64_t y = ((uint64_t)(uint32_t)pid << 32) | ((uint64_t)((uint32_t)dround & 0xFFFFu) << 16) |
               (uint64_t)((uint32_t)hround & 0xFFFFu);
  uint64_t z = ((uint64_t)(uint32_t)dec << 32) | (uint64_t)(uint32_t)mainx;
  return splitmix64(z ^ splitmix64(y));
}

// ---------------------------------------------------------------- VALU predicates
// Per-lane conditions as 0/1 integers in VGPRs. hipcc otherwise keeps every
// per-lane bool as a 64-bit SGPR lane mask and evaluates && / || with scalar
// s_and_b64/s_or_b64, which made the checker scalar-issue bound. The v_min in
// inline asm is opaque to InstCombine, so the value stays an integer.
PSG_DEV uint32_t nz01(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_min_u32 %0, %1, 1" : "=v"(r) : "v"(x));
  return r;
#else
  return x != 0;
#endif
}
PSG_DEV uint32_t ne01(int32_t a, int32_t b) { return nz01((uint32_t)(a ^ b)); }
PSG_DEV uint32_t eq01(int32_t a, int32_t b) { return 1u - nz01((uint32_t)(a ^ b)); }
PSG_DEV uint32_t gt01(int32_t a, int32_t b) { return (uint32_t)(((int64_t)b - (int64_t)a) >> 63) & 1u; }  // a > b

// OR of a per-lane word over the wave (DPP row_shr 1/2/4/8, row_bcast 15/31),
// returned as a uniform value (read from lane 63).
// Lane l receives lane l ^ D's v, without the LDS crossbar: D = 1, 2 one DPP quad_perm;
// D = 4, 8 a DPP row shift each way and a select; D = 16, 32 one v_permlane16/32_swap (a
// half exchange of v with itself) and a select.
// PSG_XSHFL_MASK: the distances D (bit log2 D) done in registers, the others by ds_bpermute.
// Default none: on the VALU-bound Epsilon sort + transposes (W2 row) all-register measured
// 18.1 ms, D = 16 / 32 only 16.1, D = 1 / 2 only 15.2, ds_bpermute for all 15.2 (the LDS
// crossbar runs beside the VALU; the register forms cost 1-3 VALU per dword).
#ifndef PSG_XSHFL_MASK
#define PSG_XSHFL_MASK 0
#endif
template <int D>
PSG_DEV uint32_t xshfl(uint32_t v, int lane) {
  static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "xor distance");
  if constexpr (((PSG_XSHFL_MASK >> __builtin_ctz(D)) & 1) == 0) return (uint32_t)__shfl_xor((int)v, D);
  else if constexpr (D == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (D == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (D == 4 || D == 8) {
    const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 + D, 0xF, 0xF, false);  // row_shl:D
    const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + D, 0xF, 0xF, false);  // row_shr:D
    return (lane & D) ? dn : up;
  } else if constexpr (D == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // odd rows <- even rows of v
    return (lane & 16) ? (uint32_t)r[0] : (uint32_t)r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);  // upper half <- lower half of v
    return (lane & 32) ? (uint32_t)r[0] : (uint32_t)r[1];
  }
}
template <int D>
PSG_DEV uint64_t xshfl64(uint64_t v, int lane) {
  return (uint64_t)xshfl<D>((uint32_t)v, lane) | ((uint64_t)xshfl<D>((uint32_t)(v >> 32), lane) << 32);
}

PSG_DEV uint32_t wave_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// ---------------------------------------------------------------- masks
template <int W>
struct Mask {
  uint64_t w[W];
};

template <int W>
PSG_DEV Mask<W> mzero() {
  Mask<W> m;
#pragma unroll
  for (int i = 0; i < W; ++i) m.w[i] = 0;
  return m;
}
template <int W>
PSG_DEV Mask<W> mand(const Mask<W>& a, const Mask<W>& b) {
  Mask<W> m;
#pragma unroll
  for (int i = 0; i < W; ++i) m.w[i] = a.w[i] & b.w[i];
  return m;
}
template <int W>
PSG_DEV Mask<W> mandn(const Mask<W>& a, const Mask<W>& b) {  // a & ~b
  Mask<W> m;
#pragma unroll
  for (int i = 0; i < W; ++i) m.w[i] = a.w[i] & ~b.w[i];
  return m;
}
template <int W>
PSG_DEV Mask<W> mor(const Mask<W>& a, const Mask<W>& b) {
  Mask<W> m;
#pragma unroll
  for (int i = 0; i < W; ++i) m.w[i] = a.w[i] | b.w[i];
  return m;
}
template <int W>
PSG_DEV int mpopc(const Mask<W>& a) {
  int c = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) c += __popcll(a.w[i]);
  return c;
}
template <int W>
PSG_DEV bool many(const Mask<W>& a) {
  uint64_t o = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) o |= a.w[i];
  return o != 0;
}
template <int W>
PSG_DEV bool meq(const Mask<W>& a, const Mask<W>& b) {
  uint64_t o = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) o |= a.w[i] ^ b.w[i];
  return o == 0;
}
template <int W>
PSG_DEV bool mtest(const Mask<W>& a, int q) {
  // an AND with a per-word bit (not a word select: LLVM turns a select chain over a
  // uniform index back into a private-array load, i.e. a scratch round trip)
  if (W == 1) return (a.w[0] >> (q & 63)) & 1ull;
  const uint64_t bit = 1ull << (q & 63);
  uint64_t hit = 0;
#pragma unroll
  for (int i = 0; i < W; ++i) hit |= a.w[i] & (((q >> 6) == i) ? bit : 0ull);
  return hit != 0;
}
template <int W>
PSG_DEV void mset(Mask<W>& a, int q) {
#pragma unroll
  for (int i = 0; i < W; ++i)
    if ((q >> 6) == i) a.w[i] |= 1ull << (q & 63);
}
template <int W>
PSG_DEV void mclear(Mask<W>& a, int q) {
#pragma unroll
  for (int i = 0; i < W; ++i)
    if ((q >> 6) == i) a.w[i] &= ~(1ull << (q & 63));
}
// first set pid (-1 if empty)
template <int W>
PSG_DEV int mfirst(const Mask<W>& a) {
#pragma unroll
  for (int i = 0; i < W; ++i)
    if (a.w[i]) return i * 64 + __builtin_ctzll(a.w[i]);
  return -1;
}
// last set pid (-1 if empty)
template <int W>
PSG_DEV int mlast(const Mask<W>& a) {
#pragma unroll
  for (int i = W - 1; i >= 0; --i)
    if (a.w[i]) return i * 64 + 63 - __builtin_clzll(a.w[i]);
  return -1;
}
template <int W>
PSG_DEV Mask<W> mfull(int n) {
  Mask<W> m;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    const int lo = i * 64;
    m.w[i] = n >= lo + 64 ? ~0ull : (n <= lo ? 0ull : ((1ull << (n - lo)) - 1ull));
  }
  return m;
}

// A uniform value moved into a VGPR: the compiler treats the result as divergent, so the
// arithmetic on it issues on the vector pipe. For the kernels bound by scalar issue (one SALU
// instruction per cycle per CU, shared by every wave of the CU) against two VALU per cycle.
PSG_DEV uint32_t vgpr_u32(uint32_t v) {
  asm("; vgpr_u32" : "+v"(v));
  return v;
}
// popcount of a mask on the vector pipe (v_bcnt), as a uniform value in a VGPR
template <int W>
PSG_DEV int mpopc_v(const Mask<W>& a) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < W; ++i)
    c += (uint32_t)__builtin_popcount(vgpr_u32((uint32_t)a.w[i])) + (uint32_t)__builtin_popcount(vgpr_u32((uint32_t)(a.w[i] >> 32)));
  return (int)c;
}

PSG_DEV uint64_t rfl64(uint64_t v) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
PSG_DEV int32_t rfl32(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
PSG_DEV int32_t readlane32(int32_t v, int q) { return __builtin_amdgcn_readlane(v, q); }
PSG_DEV uint64_t readlane64(uint64_t v, int q) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, q);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), q);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// ---------------------------------------------------------------- group of W waves = one instance
// LDS per group (W > 1): ballot ping-pong [2][W] + reduction scratch [W] + staged
// per-process arrays. For W == 1 everything stays in registers (readlane).
// First element of a pid set in Scala Map iteration order, for a per-lane set
// (every receiver has its own mailbox). CHAMP pre-order: at each trie level the
// payload entries (fragments holding exactly one element) come first in
// ascending fragment order, then the sub-nodes; so the head is the payload with
// the smallest fragment at the first level that has one, after descending into
// the smallest multi-element fragment. ChampTable holds, per level l and
// fragment f, the mask of pids whose improve(pid) has fragment f at level l.
template <int W>
struct ChampTable {
  uint64_t b[7][32][W];
  // once per block
  PSG_DEV void build(int n) {
    for (int e = threadIdx.x; e < 7 * 32 * W; e += blockDim.x) {
      const int l = e / (32 * W), f = (e / W) % 32, w = e % W;
      uint64_t m = 0;
      for (int j = 0; j < 64; ++j) {
        const int q = w * 64 + j;
        if (q < n && ((scala_improve((uint32_t)q) >> (5 * l)) & 31u) == (uint32_t)f) m |= 1ull << j;
      }
      b[l][f][w] = m;
    }
  }
};

template <int W>
PSG_DEV int champ_first(const ChampTable<W>& T, Mask<W> cur, int tiebreak) {
  const int m = mpopc(cur);
  if (m == 0) return -1;
  if (tiebreak == PSG_TIE_MIN_PID || m <= 4) return mfirst(cur);  // Map1..Map4: insertion order
  for (int l = 0; l < 7; ++l) {
    int sub = -1;
    for (int f = 0; f < 32; ++f) {
      Mask<W> e;
#pragma unroll
      for (int w = 0; w < W; ++w) e.w[w] = cur.w[w] & T.b[l][f][w];
      const int pc = mpopc(e);
      if (pc == 1) return mfirst(e);
      if (pc >= 2 && sub < 0) sub = f;
    }
#pragma unroll
    for (int w = 0; w < W; ++w) cur.w[w] &= T.b[l][sub][w];
  }
  return mfirst(cur);  // unreachable: hashes of distinct pids differ
}

template <int W>
struct Grp {
  int lane;   // 0..63
  int wv;     // wave index inside the instance
  int pid;    // wv * 64 + lane
  bool valid; // pid < n
  int ph;
  uint64_t vmask;  // uniform: valid lanes of this wave
  uint64_t* xb;  // LDS: [2][W] ballot words
  int64_t* red;  // LDS: [2][W] reduction words

  PSG_DEV void sync() const {
    if constexpr (W > 1) __syncthreads();
  }

  // LDS words of the ballot exchange (xb): two alternating regions of kFuse x W words,
  // so a region is rewritten only after the next barrier.
  static constexpr int kFuse = 6;
  static constexpr int kXb = 2 * kFuse * W;

  // Mask of the processes for which pred holds (pred is ANDed with valid).
  PSG_DEV Mask<W> ballot(bool pred) {
    const uint64_t b = __builtin_amdgcn_ballot_w64(pred) & vmask;
    Mask<W> m;
    if constexpr (W == 1) {
      m.w[0] = b;
    } else {
      uint64_t* s = xb + ph * kFuse * W;
      ph ^= 1;
      if (lane == 0) s[wv] = b;
      __syncthreads();
#pragma unroll
      for (int i = 0; i < W; ++i) m.w[i] = rfl64(s[i]);
    }
    return m;
  }
  // K ballots over one barrier (W > 1: one LDS exchange instead of K).
  template <int K>
  PSG_DEV void ballots(const bool (&pred)[K], Mask<W> (&m)[K]) {
    static_assert(K <= kFuse, "ballots: at most kFuse predicates");
    uint64_t b[K];
#pragma unroll
    for (int j = 0; j < K; ++j) b[j] = __builtin_amdgcn_ballot_w64(pred[j]) & vmask;
    if constexpr (W == 1) {
#pragma unroll
      for (int j = 0; j < K; ++j) m[j].w[0] = b[j];
    } else {
      uint64_t* s = xb + ph * kFuse * W;
      ph ^= 1;
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < K; ++j) s[j * W + wv] = b[j];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int i = 0; i < W; ++i) m[j].w[i] = rfl64(s[j * W + i]);
      }
    }
  }
  PSG_DEV bool any(bool pred) { return many(ballot(pred)); }
  // any() for predicates that are false on every lane past n (no valid-lane mask)
  PSG_DEV bool any_raw(bool pred) { return many(ballot_any(pred)); }
  // ballot() without the valid-lane mask (W == 1: one compare, no scalar AND); for
  // callers that only intersect the result with masks of valid processes
  PSG_DEV Mask<W> ballot_any(bool pred) {
    if constexpr (W == 1) {
      Mask<W> m;
      m.w[0] = __builtin_amdgcn_ballot_w64(pred);
      return m;
    } else {
      return ballot(pred);
    }
  }

  // value of process q (uniform q): W==1 readlane of `mine`; W>1 from a staged LDS array.
  PSG_DEV int32_t bcast(int32_t mine, const int32_t* staged, int q) const {
    if constexpr (W == 1) return readlane32(mine, q);
    else return rfl32(staged[q]);
  }

  // value of process q for a per-lane q (call from converged code): W==1 a
  // ds_bpermute of `mine`; W>1 from a staged LDS array.
  PSG_DEV int32_t gather(int32_t mine, const int32_t* staged, int q) const {
    if constexpr (W == 1) return __shfl(mine, q);
    else return staged[q];
  }

  // group reductions over valid lanes (inactive lanes contribute the identity).
  // Wave part: DPP row_shr 1/2/4/8 + row_bcast 15/31 (VALU latency, no LDS-crossbar
  // round trips), the result read from lane 63 as a uniform value; call from
  // converged control flow (every lane of the wave active).
  template <int CTRL, int RM>
  PSG_DEV static int32_t dpp32(int32_t old, int32_t v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xF, false);
  }
  template <int CTRL, int RM>
  PSG_DEV static int64_t dpp64(int64_t old, int64_t v) {
    const uint32_t lo = (uint32_t)dpp32<CTRL, RM>((int32_t)(uint32_t)old, (int32_t)(uint32_t)v);
    const uint32_t hi = (uint32_t)dpp32<CTRL, RM>((int32_t)(old >> 32), (int32_t)(v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  }
  template <bool MAX>
  PSG_DEV static int32_t dpp_reduce32(int32_t v) {
    constexpr int32_t id = MAX ? INT32_MIN : INT32_MAX;
#define PSG_RED32(C, R) { const int32_t t = dpp32<C, R>(id, v); v = MAX ? (t > v ? t : v) : (t < v ? t : v); }
    PSG_RED32(0x111, 0xF) PSG_RED32(0x112, 0xF) PSG_RED32(0x114, 0xF) PSG_RED32(0x118, 0xF)
    PSG_RED32(0x142, 0xA) PSG_RED32(0x143, 0xC)
#undef PSG_RED32
    return __builtin_amdgcn_readlane(v, 63);
  }
  template <bool MAX>
  PSG_DEV static int64_t dpp_reduce64(int64_t v) {
    constexpr int64_t id = MAX ? INT64_MIN : INT64_MAX;
#define PSG_RED64(C, R) { const int64_t t = dpp64<C, R>(id, v); v = MAX ? (t > v ? t : v) : (t < v ? t : v); }
    PSG_RED64(0x111, 0xF) PSG_RED64(0x112, 0xF) PSG_RED64(0x114, 0xF) PSG_RED64(0x118, 0xF)
    PSG_RED64(0x142, 0xA) PSG_RED64(0x143, 0xC)
#undef PSG_RED64
    return (int64_t)readlane64((uint64_t)v, 63);
  }
  // sum of a per-lane 32-bit value over the wave (DPP inclusive scan, total in lane 63)
  PSG_DEV static uint32_t wave_sum32(uint32_t v) {
#define PSG_SUM32(C, R) v += (uint32_t)dpp32<C, R>(0, (int32_t)v);
    PSG_SUM32(0x111, 0xF) PSG_SUM32(0x112, 0xF) PSG_SUM32(0x114, 0xF) PSG_SUM32(0x118, 0xF)
    PSG_SUM32(0x142, 0xA) PSG_SUM32(0x143, 0xC)
#undef PSG_SUM32
    return (uint32_t)__builtin_amdgcn_readlane((int32_t)v, 63);
  }
  PSG_DEV int64_t wave_min64(int64_t v) const { return dpp_reduce64<false>(v); }
  PSG_DEV int64_t wave_max64(int64_t v) const { return dpp_reduce64<true>(v); }
  PSG_DEV uint64_t wave_sum64(uint64_t v) const {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
  }
  PSG_DEV int32_t wave_min32(int32_t v) const { return dpp_reduce32<false>(v); }
  PSG_DEV int32_t wave_max32(int32_t v) const { return dpp_reduce32<true>(v); }
  template <int OP>  // 0 min, 1 max, 2 sum, 3 or
  PSG_DEV int64_t cross64(int64_t v) {
    if constexpr (W == 1) {
      return v;
    } else {
      int64_t* s = red + ph * W;
      ph ^= 1;
      if (lane == 0) s[wv] = v;
      __syncthreads();
      int64_t r = s[0];
#pragma unroll
      for (int i = 1; i < W; ++i) {
        int64_t t = s[i];
        if (OP == 0) r = t < r ? t : r;
        else if (OP == 1) r = t > r ? t : r;
        else if (OP == 2) r = (int64_t)((uint64_t)r + (uint64_t)t);
        else r = r | t;
      }
      return r;
    }
  }
  // OR of a per-lane word over the group (uniform result)
  PSG_DEV uint32_t gor(uint32_t v) {
    const uint32_t w = wave_or(v);
    if constexpr (W == 1) {
      return w;
    } else {
      return (uint32_t)cross64<3>((int64_t)w);
    }
  }
  PSG_DEV int64_t min64(int64_t v, bool in) { return cross64<0>(wave_min64((in && valid) ? v : INT64_MAX)); }
  PSG_DEV int64_t max64(int64_t v, bool in) { return cross64<1>(wave_max64((in && valid) ? v : INT64_MIN)); }
  PSG_DEV uint64_t sum64(uint64_t v) { return (uint64_t)cross64<2>((int64_t)wave_sum64(valid ? v : 0)); }
  PSG_DEV int32_t min32(int32_t v, bool in) {
    int32_t m = wave_min32((in && valid) ? v : INT32_MAX);
    if constexpr (W == 1) return m;
    else return (int32_t)cross64<0>(m);
  }
  // min32 over the `in` lanes and the group OR of `flag` in one exchange
  PSG_DEV int32_t min32_any(int32_t v, bool in, bool flag, bool& any) {
    const int32_t m = wave_min32((in && valid) ? v : INT32_MAX);
    const bool f = (__builtin_amdgcn_ballot_w64(flag) & vmask) != 0ull;
    if constexpr (W == 1) {
      any = f;
      return m;
    } else {
      int64_t* s = red + ph * W;
      ph ^= 1;
      if (lane == 0) s[wv] = ((int64_t)(f ? 1 : 0) << 32) | (int64_t)(uint32_t)m;
      __syncthreads();
      int32_t r = INT32_MAX;
      bool a = false;
#pragma unroll
      for (int i = 0; i < W; ++i) {
        const int64_t t = s[i];
        const int32_t ti = (int32_t)(uint32_t)t;
        r = ti < r ? ti : r;
        a = a || (t >> 32) != 0;
      }
      any = a;
      return r;
    }
  }
  PSG_DEV int32_t max32(int32_t v, bool in) {
    int32_t m = wave_max32((in && valid) ? v : INT32_MIN);
    if constexpr (W == 1) return m;
    else return (int32_t)cross64<1>(m);
  }
};

// Make this group's LDS writes visible to the whole group (W > 1: block barrier;
// W == 1: the wave's own LDS operations are ordered, so a wave-scope fence suffices).
template <int W>
PSG_DEV void lds_sync() {
  if constexpr (W > 1) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------- instance queue
// Dynamic distribution of a batch's instances over the resident groups.
// A static grid-stride split left the chip 30% idle on the headline launch: a
// SIMD issues by wave age, so its six resident waves run at very different
// speeds (timer build, profiles/s2_queue: the oldest wave of a SIMD finishes at
// 0.45 of the kernel span, the youngest at 1.0, in six steps), and each SIMD
// ran the second half of the launch with fewer and fewer waves to hide latency.
// Here a group takes kChunk consecutive instances at a time from one of
// NQUEUES counters (queue = blockIdx % NQUEUES, which spreads the atomics over
// the XCDs the blocks are dispatched to round-robin; queue q owns the slice
// [q*count/NQUEUES, (q+1)*count/NQUEUES)) and moves to the next queue when its
// own is drained, so every group works until the whole batch is done. Which
// group runs an instance does not change any result: per-instance outputs are
// indexed by the instance's batch row, counters are integer sums.
// The counters live in a.counters[C_QUEUE + q*QUEUE_STRIDE], zeroed before
// every launch together with the result counters.
#ifndef PSG_QUEUE_CHUNK_WIDE
#define PSG_QUEUE_CHUNK_WIDE 4  // W > 1 (one instance per block): 1 -> 4 measured +2-4 % on C4/C5
#endif
#ifndef PSG_QUEUE_CHUNK
#define PSG_QUEUE_CHUNK 4
#endif
// OTR / OTR2, LastVoting, ShortLastVoting at W = 1 (CHUNK argument): 4 -> 8 measured headline
// 19.24 -> 19.08 ms, C3 46.88 -> 46.78 (round 6); the packed kernels and Epsilon lost 1-4 % at 8
#ifndef PSG_QUEUE_CHUNK_LANE
#define PSG_QUEUE_CHUNK_LANE 8
#endif
template <int W, int REGION = 0, int CHUNK = 0>
struct InstanceQueue {
  static_assert(REGION >= 0 && REGION < NQUEUE_REGIONS, "queue region");
  static constexpr uint64_t kChunk = CHUNK > 0 ? CHUNK : (W == 1 ? PSG_QUEUE_CHUNK : PSG_QUEUE_CHUNK_WIDE);
  static constexpr uint64_t kDone = ~0ull;
  uint64_t cur = 0, lim = 0;  // uniform: [cur, lim) is this group's current chunk
  int tries = 0;              // queues drained so far

  // Next batch row of this group, kDone when the whole batch is taken.
  // Called by every lane of the group in converged control flow.
  PSG_DEV uint64_t take(const KArgs& a) {
    if (cur < lim) return cur++;
    const int home = (int)(blockIdx.x % NQUEUES);
    for (; tries < NQUEUES; ++tries) {
      const int q = (home + tries) % NQUEUES;
      const uint64_t lo = a.count * q / NQUEUES, hi = a.count * (q + 1) / NQUEUES;
      if (lo >= hi) continue;
      const uint64_t v = grab(&a.counters[C_QUEUE + (REGION * NQUEUES + q) * QUEUE_STRIDE]);
      if (lo + v < hi) {
        cur = lo + v;
        lim = cur + kChunk < hi ? cur + kChunk : hi;
        return cur++;
      }
    }
    return kDone;
  }

 private:
  // one atomic per group, its old value broadcast to every lane of the group
  PSG_DEV static uint64_t grab(unsigned long long* c) {
    if constexpr (W == 1) {
      uint64_t v = 0;
      if ((threadIdx.x & 63) == 0) v = atomicAdd(c, (unsigned long long)kChunk);
      return rfl64(v);
    } else {
      __shared__ uint64_t slot;
      if (threadIdx.x == 0) slot = atomicAdd(c, (unsigned long long)kChunk);
      __syncthreads();
      const uint64_t v = rfl64(slot);
      __syncthreads();  // slot is rewritten by the next grab
      return v;
    }
  }
};

// ---------------------------------------------------------------- schedule
// XHO: explicit schedule (psg_load_schedule) — HO sets read from HBM instead of
// drawn; a separate instantiation so the seeded hot path keeps its registers.
template <int W, bool XHO = false>
struct Sched {
  uint64_t seed, inst;
  Mask<W> full;
  int32_t crash_round;  // this process's crash round, -1 = correct
  bool crash_on;
  int good_min, ho_min, V;
  uint32_t drop, good_p32, self_bit;
  int nproc;
  const uint64_t* hop;  // explicit schedule of this instance ([R][n][W] words), or null

  PSG_DEV void setup(const KArgs& args, uint64_t i, int pid, bool valid) {
    hop = nullptr;
    nproc = args.n;
    if constexpr (XHO) {  // explicit schedule: HO sets read verbatim, no seeded draws
      const uint64_t row = i - args.ho_base;
      hop = args.ho_in + row * (uint64_t)args.R * (uint64_t)args.n * W;
      seed = args.seed;
      inst = i;
      V = args.V;
      drop = 0;
      good_p32 = 0;
      self_bit = 0;
      ho_min = -1;
      full = mfull<W>(args.n);
      crash_on = false;
      good_min = 0;
      crash_round = (args.crash_in && valid) ? args.crash_in[row * (uint64_t)args.n + pid] : -1;
      return;
    }
    seed = args.seed;
    inst = i;
    V = args.V;
    drop = args.drop_log2;
    good_p32 = args.good_p32;
    self_bit = args.self_bit;
    ho_min = args.ho_min;
    full = mfull<W>(args.n);
    crash_on = args.crash_fmax >= 0;
    good_min = args.good_min >= 0 ? args.good_min : (2 * args.n) / 3;
    crash_round = -1;
    if (crash_on && valid) {
      const uint64_t w0 = rword(seed, i, ROUND_CRASH, PID_GLOBAL, 0);
      const uint64_t w1 = rword(seed, i, ROUND_CRASH, PID_GLOBAL, 1);
      crash_round = crash_of(args, i, (uint32_t)pid, w0, w1);
    }
  }

  // Crash round of process pid (-1 = correct) from the instance's two crash words
  // w0, w1 (round ROUND_CRASH, pid PID_GLOBAL, words 0 and 1): f = the number of
  // crashed processes, an affine permutation of the pids picks them.
  PSG_DEV static int32_t crash_of(const KArgs& args, uint64_t i, uint32_t pid, uint64_t w0, uint64_t w1) {
    const uint32_t f = mulhi32((uint32_t)w0, (uint32_t)args.crash_fmax + 1u);
    const uint32_t am = (uint32_t)(w0 >> 32) | 1u;
    const uint32_t off = (uint32_t)w1;
    const uint32_t n = (uint32_t)args.n;
    const bool pow2 = (n & (n - 1)) == 0;
    const uint32_t pos = pow2 ? ((am * pid + off) & (n - 1)) : ((pid + off % n) % n);
    if (pos >= f) return -1;
    return (int32_t)mulhi32((uint32_t)rword(args.seed, i, ROUND_CRASH, pid, 0), (uint32_t)args.R);
  }

  PSG_DEV int32_t init_value(int pid, int alg) const {
    const uint64_t w = rword(seed, inst, ROUND_INIT, (uint32_t)pid, 0);
    if (alg == PSG_ALG_BENOR) return (int32_t)((uint32_t)w & 1u);
    return 1 + (int32_t)mulhi32((uint32_t)w, (uint32_t)V);
  }

  PSG_DEV bool coin(int k, int pid) const {
    return java_first_boolean(rword(seed, inst, (uint32_t)k, COIN_TAG | (uint32_t)pid, 0));
  }

  // Good rounds are uniform per (instance, round). Lane l of every wave draws
  // round base + l in parallel (one vector Philox pass per 64 rounds) instead of
  // a scalar-dependent draw per round; the flags become one 64-bit ballot.
  uint64_t good_mask;
  int good_base;
  Mask<W> good_set;  // lane l: common HO set of round good_base + l

  PSG_DEV void prep_good(int kbase, int lane, int R) {
    good_base = kbase;
    good_mask = 0;
    if (good_p32 == 0) return;
    const int k = kbase + lane;
    WordStream ws(seed, inst, (uint32_t)k, PID_GLOBAL);
    const bool good = k < R && (uint32_t)ws.word(0) < good_p32;
    Mask<W> s = full;
    if (good && drop > 0) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t m = ~0ull;
        for (uint32_t i = 0; i < drop; ++i) m &= ws.word(1u + (uint32_t)w * drop + i);
        s.w[w] &= ~m;
      }
      if (mpopc(s) <= good_min) s = full;
    }
    good_set = s;
    good_mask = __builtin_amdgcn_ballot_w64(good);
  }

  PSG_DEV bool good_round(int k, int lane, int R, Mask<W>& s) {
    if (good_p32 == 0) return false;  // no good rounds in this launch (one scalar test per round)
    if (k - good_base >= 64) prep_good(k, lane, R);
    const int off = k - good_base;
    const bool good = (good_mask >> off) & 1ull;
    if (good) {
#pragma unroll
      for (int w = 0; w < W; ++w) s.w[w] = readlane64(good_set.w[w], off);
    }
    return good;
  }

  // Raw random words of HO(pid) in round k, drawn in one straight-line pass over
  // the Philox calls of pid's stream (no divergent word cache): word j < W*drop
  // feeds drop mask j / drop (dm[w] = AND of word w's drop words), word W*drop + w
  // is the crash-round survival mask hf[w] of word w. good: the drop words are not
  // needed (the round's common set replaces them); crash = false: the survival
  // words are not needed (no process crashes in round k) and hf stays all-ones.
  // cw (uniform): bit w set iff survival word w is needed (some process of pid word w crashes in
  // round k); a call whose two words are neither drop words nor needed survival words is skipped
  // (those survival words are only ever ANDed with an empty CN word: packed KSet at n = 256
  // draws one call instead of two in most crash rounds).
  // Words j0 .. j1 - 1 of pid's stream in round k into dm / hf; SKIP: a call whose two words are
  // neither drop words nor survival words of a non-empty CN word (cw) is skipped.
  template <bool SKIP>
  PSG_DEV void draw_words(uint32_t k, uint32_t pid, uint32_t j0, uint32_t j1, uint32_t nd, uint32_t cw,
                          uint64_t (&dm)[W], uint64_t (&hf)[W]) const {
    for (uint32_t sidx = j0 >> 1; 2 * sidx < j1; ++sidx) {
      if constexpr (SKIP) {
        bool need = false;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t j = 2 * sidx + (uint32_t)h;
          need = need || (j >= j0 && j < j1 && (j < nd || ((cw >> (j - nd)) & 1u)));
        }
        if (!need) continue;
      }
      const U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), k, pid + (sidx << 16), (uint32_t)seed,
                            (uint32_t)(seed >> 32));
      const uint64_t wlo = (uint64_t)o.x | ((uint64_t)o.y << 32);
      const uint64_t whi = (uint64_t)o.z | ((uint64_t)o.w << 32);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t j = 2 * sidx + (uint32_t)h;
        const uint64_t word = h ? whi : wlo;
        if (j < j0 || j >= j1) continue;
        if (j < nd) {
          const uint32_t wi = j / drop;
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (wi == (uint32_t)w) dm[w] &= word;
        } else {
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (j - nd == (uint32_t)w) hf[w] = word;
        }
      }
    }
  }
  // SKIP = false: the plain loop (BenOr: the skip test in every call measured 9 % slower on its
  // crash-free C5 rows, a skip-only-in-crash-rounds second loop 2.5 % slower on packed KSet;
  // round-4 A/Bs)
  template <bool SKIP = true>
  PSG_DEV void draw(uint32_t k, uint32_t pid, bool good, bool crash, uint64_t (&dm)[W], uint64_t (&hf)[W],
                    uint32_t cw = ~0u) const {
    const uint32_t nd = (uint32_t)W * drop;
    const uint32_t j0 = good ? nd : 0u;
    const uint32_t j1 = crash ? nd + (uint32_t)W : (good ? 0u : nd);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      dm[w] = ~0ull;
      hf[w] = ~0ull;
    }
    constexpr bool kSkip = SKIP && W > 1;
    if constexpr (kSkip) {
      // loss-free schedules (C4) in crash rounds: only the survival words, W / 2 unrolled calls
      // instead of the runtime-bounded word loop (packed KSet f = 64 7.63 -> 6.32 ms, KSetES -5.5 %,
      // f = 1 +3.5 %: round-4 A/B)
      if (__builtin_expect(drop == 0 && crash, 0)) {  // (laid out of line: packed KSet -1.5 %)
        {
#pragma unroll
          for (int sc2 = 0; 2 * sc2 < W; ++sc2) {
            if (!((cw >> (2 * sc2)) & 3u)) continue;  // neither word's 64 pids crash in round k
            const U4 o = philox10((uint32_t)inst, (uint32_t)(inst >> 32), k, pid + ((uint32_t)sc2 << 16),
                                  (uint32_t)seed, (uint32_t)(seed >> 32));
            hf[2 * sc2] = (uint64_t)o.x | ((uint64_t)o.y << 32);
            if (2 * sc2 + 1 < W) hf[2 * sc2 + 1] = (uint64_t)o.z | ((uint64_t)o.w << 32);
          }
        }
        return;
      }
    }
    draw_words<kSkip>(k, pid, j0, j1, nd, cw, dm, hf);
  }

  // HO(pid) from its raw words. CB = processes crashed before round k, CN =
  // crashing in round k (uniform).
  PSG_DEV Mask<W> assemble(int pid, bool good, const Mask<W>& goodS, const Mask<W>& CB, const Mask<W>& CN,
                           const uint64_t (&dm)[W], const uint64_t (&hf)[W]) const {
    Mask<W> base;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      base.w[w] = good ? goodS.w[w] : (drop > 0 ? full.w[w] & ~dm[w] : full.w[w]);
      if (crash_on) base.w[w] &= ~(CB.w[w] | (CN.w[w] & ~hf[w]));
    }
    if (self_bit) mset(base, pid);
    if (ho_min >= 0 && mpopc(base) <= ho_min) base = full;
    return base;
  }

  // HO(p) for this lane's process p in round k.
  template <bool SKIP = true>
  PSG_DEV Mask<W> ho(int k, int pid, bool good, const Mask<W>& goodS, const Mask<W>& CB, const Mask<W>& CN) const {
    if constexpr (XHO) {  // explicit: W contiguous words per process, the wave reads 512*W contiguous bytes
      Mask<W> m = mzero<W>();
      if (pid < nproc) {
        const uint64_t* q = hop + ((uint64_t)k * (uint64_t)nproc + (uint64_t)pid) * W;
#pragma unroll
        for (int w = 0; w < W; ++w) m.w[w] = __builtin_nontemporal_load(q + w) & full.w[w];
      }
      return m;
    }
    uint64_t dm[W], hf[W];
    uint32_t cw = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) cw |= CN.w[w] ? 1u << w : 0u;
    draw<SKIP>((uint32_t)k, (uint32_t)pid, good, crash_on && cw != 0u, dm, hf, cw);
    return assemble(pid, good, goodS, CB, CN, dm, hf);
  }
};

// Crash sets of round k: CB = processes crashed before round k, CN = crashing in
// round k. A process's crash round is fixed per instance, so for W > 1 the
// instance's crash rounds are staged in LDS once (one barrier per instance) and
// lane l keeps those of processes w*64 + l in registers: every wave then forms
// CB(k) / CN(k) from 2W local ballots, with no per-round cross-wave exchange.
// W == 1: the two ballots are already wave-local.
template <int W>
struct CrashSets {
  int32_t cr[W];
  // lds: 64*W words (W > 1); call from uniform control flow (block barrier)
  PSG_DEV void prep(Grp<W>& g, int32_t* lds, int32_t my_crash_round) {
    if constexpr (W == 1) {
      cr[0] = my_crash_round;
    } else {
      lds[g.pid] = g.valid ? my_crash_round : -1;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < W; ++w) cr[w] = lds[w * 64 + g.lane];
    }
  }
  PSG_DEV void sets(Grp<W>& g, int k, Mask<W>& CB, Mask<W>& CN) const {
    // crashed before round k: 0 <= cr < k, one unsigned compare (cr = -1: correct)
    if constexpr (W == 1) {  // (lanes past n have crash round -1: no valid-lane mask needed)
      CB = g.ballot_any((uint32_t)cr[0] < (uint32_t)k);
      CN = g.ballot_any(cr[0] == k);
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        CB.w[w] = __builtin_amdgcn_ballot_w64((uint32_t)cr[w] < (uint32_t)k);
        CN.w[w] = __builtin_amdgcn_ballot_w64(cr[w] == k);
      }
    }
  }
};

// ---------------------------------------------------------------- per-instance checks
struct Checks {
  // One VGPR: lane s (< PSG_MAX_CHECKS) holds slot s's first failing check point, lane
  // PSG_MAX_CHECKS the first check point where Termination holds (PSG_NEVER: none). Check
  // points arrive in increasing order, so "first" is a running minimum, and recording is
  // branch-free per-lane VALU work (no scalar state: the kernels are scalar-issue-bound).
  int32_t ffv;
  PSG_DEV void reset() { ffv = PSG_NEVER; }
  // failbits: bit s set iff slot s is false at check point c (uniform); term: Termination holds
  PSG_DEV void record(uint32_t failbits, bool term, int c, int lane) {
    const uint32_t bits = failbits | (term ? (1u << PSG_MAX_CHECKS) : 0u);
    // lane's bit of the 13-bit word (a 32-bit shift reads only the amount's low 5 bits: lanes
    // past PSG_MAX_CHECKS take the all-zero mask instead, one AND + compare per check point)
    const uint32_t mine = lane <= PSG_MAX_CHECKS ? 1u << lane : 0u;
    const int32_t at = (bits & mine) ? c : (int32_t)PSG_NEVER;
    ffv = at < ffv ? at : ffv;
  }
  // slot `lane` (< PSG_MAX_CHECKS) failed at some check point
  PSG_DEV bool failed_here() const { return ffv != (int32_t)PSG_NEVER; }
  PSG_DEV uint32_t term_round() const { return (uint32_t)__builtin_amdgcn_readlane(ffv, PSG_MAX_CHECKS); }
};

PSG_DEV uint32_t fbit(bool ok, int slot) { return ok ? 0u : (1u << slot); }

// Block-level accumulators in LDS, flushed once per block.
struct BlockCounters {
  unsigned int fail[PSG_MAX_CHECKS];
  unsigned int decided;
  unsigned int hist[PSG_MAX_ROUNDS + 2];
  unsigned long long digest;
  unsigned long long active, live;  // C_ACTIVE / C_LIVE partial sums
};

PSG_DEV void counters_init(BlockCounters* bc) {
  for (int i = threadIdx.x; i < PSG_MAX_CHECKS; i += blockDim.x) bc->fail[i] = 0;
  for (int i = threadIdx.x; i < PSG_MAX_ROUNDS + 2; i += blockDim.x) bc->hist[i] = 0;
  if (threadIdx.x == 0) {
    bc->decided = 0;
    bc->digest = 0;
    bc->active = 0;
    bc->live = 0;
  }
}

PSG_DEV void counters_flush(BlockCounters* bc, unsigned long long* g, int nchecks, int R) {
  for (int i = threadIdx.x; i < nchecks; i += blockDim.x)
    if (bc->fail[i]) atomicAdd(&g[C_FAIL + i], (unsigned long long)bc->fail[i]);
  for (int i = threadIdx.x; i < R + 2; i += blockDim.x)
    if (bc->hist[i]) atomicAdd(&g[C_HIST + i], (unsigned long long)bc->hist[i]);
  if (threadIdx.x == 0) {
    atomicAdd(&g[C_DECIDED], (unsigned long long)bc->decided);
    atomicAdd(&g[C_DIGEST], bc->digest);
    atomicAdd(&g[C_ACTIVE], bc->active);
    atomicAdd(&g[C_LIVE], bc->live);
  }
}

// Per-lane running sum of the process-round steps over a wave's instances (C_ACTIVE), reduced
// and flushed once per wave instead of a wave reduction per instance.
struct StepTally {
  uint64_t steps = 0;  // this lane's processes' steps over the wave's instances
  PSG_DEV void add(int32_t s) { steps += (uint64_t)(uint32_t)s; }
  // every lane of the wave, converged; one LDS atomic per wave
  PSG_DEV void flush(BlockCounters* bc) {
    Grp<1> g1;
    const uint64_t t = g1.wave_sum64(steps);
    if ((threadIdx.x & 63) == 0) atomicAdd(&bc->active, (unsigned long long)t);
  }
};

// Per-instance epilogue: digest, decide results, summaries, counters.
// Called by every lane of the group; lane values are this process's results.
// tally (optional): accumulate the steps per lane (StepTally::flush at the end of the kernel)
// instead of a wave sum per instance; live_rounds >= 0: the rounds the instance executed (some
// process active), known to the caller, instead of a wave maximum.
template <int W>
PSG_DEV void finish_instance(Grp<W>& g, const KArgs& a, uint64_t i, const Checks& ck, int nchecks, int32_t dec_val,
                             int32_t dec_round, int32_t halt_round, int32_t main_x, BlockCounters* bc,
                             StepTally* tally = nullptr, int32_t live_rounds = -1) {
  const int n = a.n;
  const bool decided = dec_round >= 0;
  const uint64_t d = g.valid ? proc_digest(g.pid, dec_val, dec_round, halt_round, main_x) : 0ull;
  const uint64_t dig = g.sum64(d);
  const int nd = mpopc(g.ballot(decided));
  // rounds in which this process took a step: up to and including its halting round
  const int32_t steps = g.valid ? (halt_round >= 0 ? halt_round + 1 : a.R) : 0;
  uint32_t wave_steps = 0;
  if (tally) tally->add(steps);
  else wave_steps = Grp<W>::wave_sum32((uint32_t)steps);
  const int32_t live = live_rounds >= 0 ? live_rounds : g.max32(steps, true);  // rounds executed for the instance
  if (g.valid) {
    const uint64_t off = i * (uint64_t)n + (uint64_t)g.pid;
    if (a.out_decision) a.out_decision[off] = dec_val;
    if (a.out_dround) a.out_dround[off] = decided ? (uint8_t)dec_round : (uint8_t)0xFF;
    if (a.out_rec) {
      psg_process_record r;
      r.decision = dec_val;
      r.decision_round = dec_round;
      r.halt_round = halt_round;
      r.final_x = main_x;
      a.out_rec[off] = r;
    }
  }
  if (g.wv == 0) {
    const uint32_t term = ck.term_round();
    if (a.out_inst) {
      uint8_t* o = reinterpret_cast<uint8_t*>(a.out_inst + i);
      if (g.lane < PSG_MAX_CHECKS) o[8 + g.lane] = (uint8_t)ck.ffv;  // first_fail[lane]
      if (g.lane == 0) {
        *reinterpret_cast<uint64_t*>(o) = dig;
        o[8 + PSG_MAX_CHECKS] = (uint8_t)term;
        o[9 + PSG_MAX_CHECKS] = (uint8_t)nchecks;
        *reinterpret_cast<uint16_t*>(o + 10 + PSG_MAX_CHECKS) = (uint16_t)nd;
      }
    }
    if (g.lane < nchecks && ck.failed_here()) atomicAdd(&bc->fail[g.lane], 1u);
    if (g.lane == 0) {
      atomicAdd(&bc->hist[term == PSG_NEVER ? a.R + 1 : term], 1u);
      atomicAdd(&bc->decided, (unsigned int)nd);
      atomicAdd(&bc->digest, (unsigned long long)dig);
      atomicAdd(&bc->live, (unsigned long long)live);
    }
  }
  if (!tally && g.lane == 0) atomicAdd(&bc->active, (unsigned long long)wave_steps);
}

// Process state at check point c for the Spec-program interpreter
// (psg_run_batch_spec): trace[i][c][field][pid], one coalesced row per field.
template <int W>
PSG_DEV void trace_put(const Grp<W>& g, const KArgs& a, uint64_t i, int c, int32_t x, int32_t decided,
                       int32_t decision, int32_t ts, int32_t ready, int32_t commit, int32_t vote, int32_t cand,
                       int32_t hosize) {
  if (!g.valid) return;
  const uint64_t n = (uint64_t)a.n;
  int32_t* t = a.trace + (i * (uint64_t)(a.R + 1) + (uint64_t)c) * PSG_NFIELDS * n + (uint64_t)g.pid;
  // only the fields the program reads (uniform tests): rows of unread fields stay unwritten
  const uint32_t m = a.trace_fields;
  if (m & (1u << PSG_FIELD_X)) t[PSG_FIELD_X * n] = x;
  if (m & (1u << PSG_FIELD_DECIDED)) t[PSG_FIELD_DECIDED * n] = decided;
  if (m & (1u << PSG_FIELD_DECISION)) t[PSG_FIELD_DECISION * n] = decision;
  if (m & (1u << PSG_FIELD_TS)) t[PSG_FIELD_TS * n] = ts;
  if (m & (1u << PSG_FIELD_READY)) t[PSG_FIELD_READY * n] = ready;
  if (m & (1u << PSG_FIELD_COMMIT)) t[PSG_FIELD_COMMIT * n] = commit;
  if (m & (1u << PSG_FIELD_VOTE)) t[PSG_FIELD_VOTE * n] = vote;
  if (m & (1u << PSG_FIELD_CANDECIDE)) t[PSG_FIELD_CANDECIDE * n] = cand;
  if (m & (1u << PSG_FIELD_HOSIZE)) t[PSG_FIELD_HOSIZE * n] = hosize;
}

// Spec hooks of the round kernels. NoHook: the built-in checks (+ the trace of
// psg_run_batch_spec). A fused Spec module (round_amd/formula.py
// compile_native(fused=True), psg_spec_native.hpp spec::SpecHook) instead
// evaluates a compiled Spec at every check point from the kernel's registers.
struct NoHook {
  static constexpr bool kFused = false;
  static constexpr int kSlots = 0;
  static constexpr uint32_t kFields = 0;  // state fields the hook's Spec reads (psg.h PSG_FIELD_*)
  template <int W>
  struct State {
    Checks ck;
    PSG_DEV State(Grp<W>&, int, int) {}
    PSG_DEV void put(int, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t, int32_t) {}
  };
};

// Is the process state of every check point needed (trace or fused Spec)? TR = false: the
// launch has no Spec-program trace (known at compile time: the instantiation the library's
// built-in-checker launches use, which then holds no trace pointers or field masks)
template <class SH, bool TR = true>
PSG_DEV bool tracing(const KArgs& a) {
  return SH::kFused || (TR && a.trace != nullptr);
}

// One check point's process state: to the fused Spec, else to the trace.
template <int W, class SH, class St>
PSG_DEV void emit_state(St& sh, const Grp<W>& g, const KArgs& a, uint64_t i, int c, int32_t x, int32_t decided,
                        int32_t decision, int32_t ts, int32_t ready, int32_t commit, int32_t vote, int32_t cand,
                        int32_t hosize, bool frozen = false) {
  if constexpr (SH::kFused) sh.put(c, x, decided, decision, ts, ready, commit, vote, cand, hosize, frozen);
  else trace_put<W>(g, a, i, c, x, decided, decision, ts, ready, commit, vote, cand, hosize);
}

// Group geometry: W == 1 -> 4 independent instances per 256-thread block;
// W > 1 -> one instance per block of 64*W threads.
template <int W>
struct Geometry {
  static constexpr int kThreads = W == 1 ? 256 : 64 * W;
  static constexpr int kGroups = W == 1 ? 4 : 1;
};

template <int W>
PSG_DEV void grp_setup(Grp<W>& g, const KArgs& a, uint64_t* xb, int64_t* red) {
  g.lane = threadIdx.x & 63;
  g.wv = W == 1 ? 0 : (threadIdx.x >> 6);
  g.pid = g.wv * 64 + g.lane;
  g.valid = g.pid < a.n;
  {
    const int lo = g.wv * 64;
    g.vmask = a.n >= lo + 64 ? ~0ull : (a.n <= lo ? 0ull : ((1ull << (a.n - lo)) - 1ull));
  }
  g.ph = 0;
  g.xb = xb;
  g.red = red;
}

// Set of an instance's initial values as an LDS open-addressing hash table
// (128 slots per 64 processes, load <= 1/2), built once per instance with one
// lane per value. Membership ("i.x == init(j.x) for some j", Validity) is then
// one or two LDS probes per lane instead of a loop over distinct values.
template <int W>
struct X0Set {
  static constexpr int kSlots = W == 1 ? 128 : (W == 2 ? 256 : 512);  // power of two >= 128 * W
  static constexpr int32_t kEmpty = INT32_MIN;
  int32_t* tab;
  bool has_empty;  // the sentinel value itself is an initial value
  // W == 1 with every initial value in [lo, lo + 64): the set is the 64-bit word bm
  // (bit v - lo), kept in registers, and membership is one shift and mask: no hash,
  // no LDS round trip (OTR / LastVoting synthetic values span {1..V}, V <= 64)
  bool bmode;
  int32_t lo;
  uint64_t bm;

  PSG_DEV static uint32_t slot(int32_t v) {
    constexpr int kBits = W == 1 ? 7 : (W == 2 ? 8 : 9);  // log2(kSlots)
    return ((uint32_t)v * 0x9E3779B1u) >> (32 - kBits);
  }
  PSG_DEV uint32_t bm_in01(int32_t v) const {
    const uint32_t d = (uint32_t)v - (uint32_t)lo;  // < 64 exactly when v - lo is in [0, 64)
    return d < 64u ? (uint32_t)(bm >> d) & 1u : 0u;
  }
  PSG_DEV void build(Grp<W>& g, int32_t* lds, int32_t x0) {
    tab = lds;
    bmode = false;
    lo = 0;
    bm = 0;
    if constexpr (W == 1) {
      const int32_t mn = g.min32(x0, true), mx = g.max32(x0, true);
      if ((int64_t)mx - (int64_t)mn < 64) {
        bmode = true;
        lo = mn;
        const uint64_t bit = g.valid ? 1ull << ((uint32_t)(x0 - mn) & 63u) : 0ull;
        bm = (uint64_t)wave_or((uint32_t)bit) | ((uint64_t)wave_or((uint32_t)(bit >> 32)) << 32);
        has_empty = false;
        return;
      }
    }
    for (int t = g.pid; t < kSlots; t += 64 * W) tab[t] = kEmpty;
    lds_sync<W>();
    if (g.valid && x0 != kEmpty) {
      uint32_t h = slot(x0);
      while (true) {
        const int32_t prev = atomicCAS(&tab[h], kEmpty, x0);
        if (prev == kEmpty || prev == x0) break;
        h = (h + 1) & (uint32_t)(kSlots - 1);
      }
    }
    has_empty = g.any(x0 == kEmpty);
    lds_sync<W>();
  }
  // Uniform: does every process selected by `sel` hold a value of the set?
  // Fast path: one ballot of "v is in neither of its two home slots"; the probe
  // loop runs only for lanes that miss both (load <= 1/2 makes that rare).
  PSG_DEV bool all_in(Grp<W>& g, const Mask<W>& sel, int32_t v) const {
    if (bmode) return !many(mand(g.ballot(bm_in01(v) == 0u), sel));
    const uint32_t h = slot(v);
    const int32_t t0 = tab[h];
    const int32_t t1 = tab[(h + 1) & (uint32_t)(kSlots - 1)];
    const Mask<W> need = mand(g.ballot(t0 != v && t1 != v), sel);
    if (!many(need)) return true;
    return !g.any(mtest(need, g.pid) && !contains(v));
  }

  // 1 unless v sits in one of its two home slots: 0 proves membership, 1 means
  // "maybe not a member" (resolve with contains / all_in). The sentinel value itself
  // always answers 1. (Exact in bitmap mode.)
  // (A branch-free form that computes both probes and selects one was measured 17 %
  // slower on the OTR headline, gpurun_out ab10: the branch on the uniform mode is cheaper.)
  PSG_DEV uint32_t maybe_out01(int32_t v) const {
    if (bmode) return 1u - bm_in01(v);
    const uint32_t h = slot(v);
    const int32_t t0 = tab[h];
    const int32_t t1 = tab[(h + 1) & (uint32_t)(kSlots - 1)];
    return (ne01(t0, v) & ne01(t1, v)) | eq01(v, kEmpty);
  }
  // maybe_out01 of two values under one test of the mode (one scalar branch, not two)
  PSG_DEV void maybe_out01_2(int32_t a, int32_t b, uint32_t& oa, uint32_t& ob) const {
    if (bmode) {
      oa = 1u - bm_in01(a);
      ob = 1u - bm_in01(b);
      return;
    }
    const uint32_t ha = slot(a), hb = slot(b);
    const int32_t a0 = tab[ha], a1 = tab[(ha + 1) & (uint32_t)(kSlots - 1)];
    const int32_t b0 = tab[hb], b1 = tab[(hb + 1) & (uint32_t)(kSlots - 1)];
    oa = (ne01(a0, a) & ne01(a1, a)) | eq01(a, kEmpty);
    ob = (ne01(b0, b) & ne01(b1, b)) | eq01(b, kEmpty);
  }
  // contains() as a VALU 0/1 integer (see nz01); same probing scheme
  PSG_DEV uint32_t contains01(int32_t v) const {
    if (bmode) return bm_in01(v);
    const uint32_t h = slot(v);
    const int32_t t0 = tab[h];
    const int32_t t1 = tab[(h + 1) & (uint32_t)(kSlots - 1)];
    const uint32_t e0 = eq01(t0, v), z0 = eq01(t0, kEmpty), e1 = eq01(t1, v), z1 = eq01(t1, kEmpty);
    uint32_t hit = e0 | ((1u - z0) & e1);
    const uint32_t done = e0 | z0 | e1 | z1;
    if (__builtin_amdgcn_ballot_w64(done == 0u) != 0ull) {
      if (done == 0u) {
        uint32_t q = (h + 2) & (uint32_t)(kSlots - 1);
        while (true) {
          const int32_t t = tab[q];
          if (t == v) { hit = 1u; break; }
          if (t == kEmpty) break;
          q = (q + 1) & (uint32_t)(kSlots - 1);
        }
      }
    }
    const uint32_t isE = eq01(v, kEmpty);
    return (isE & (has_empty ? 1u : 0u)) | ((1u - isE) & hit);
  }
  // Two adjacent slots are read unconditionally (load <= 1/2: almost every probe
  // resolves there); the probe loop runs only if some lane is still unresolved.
  PSG_DEV bool contains(int32_t v) const {
    if (bmode) return bm_in01(v) != 0u;
    const uint32_t h = slot(v);
    const int32_t t0 = tab[h];
    const int32_t t1 = tab[(h + 1) & (uint32_t)(kSlots - 1)];
    bool hit = t0 == v || (t0 != kEmpty && t1 == v);
    const bool done = t0 == v || t0 == kEmpty || t1 == v || t1 == kEmpty;
    if (__builtin_amdgcn_ballot_w64(!done) != 0ull) {
      if (!done) {
        uint32_t q = (h + 2) & (uint32_t)(kSlots - 1);
        while (true) {
          const int32_t t = tab[q];
          if (t == v) { hit = true; break; }
          if (t == kEmpty) break;
          q = (q + 1) & (uint32_t)(kSlots - 1);
        }
      }
    }
    return v == kEmpty ? has_empty : hit;
  }
};

#ifndef PSG_MAJ_BITVOTE
#define PSG_MAJ_BITVOTE 8  // W == 1: bitwise vote when at most this many bits differ (0: off)
#endif
// Candidate for a strict-majority value among the valid lanes of the group: if some
// value occurs more than n/2 times, it is returned; otherwise an arbitrary value.
// W == 1, few differing bits: a bitwise vote. A value held by more than half of the
// lanes agrees with more than half of them on every bit, so its bit b is the majority
// bit b (popcount of a ballot); bits on which every lane agrees come from the AND.
// Otherwise Boyer-Moore pair cancellation as a butterfly reduction (ds_bpermute steps).
template <int W>
PSG_DEV int32_t majority_candidate(Grp<W>& g, int32_t x) {
  if constexpr (W == 1 && PSG_MAJ_BITVOTE > 0) {
    const uint32_t u = (uint32_t)x;
    const uint32_t any1 = wave_or(g.valid ? u : 0u), any0 = wave_or(g.valid ? ~u : 0u);
    uint32_t diff = any1 & any0;  // bits set in some lane and clear in another
    if (__builtin_popcount(diff) <= PSG_MAJ_BITVOTE) {
      const int half = __popcll(g.vmask) / 2;
      uint32_t m = any1 & ~any0;  // bits set in every lane
      while (diff) {
        const int b = __builtin_ctz(diff);
        diff &= diff - 1u;
        if (__popcll(__builtin_amdgcn_ballot_w64((u >> b) & 1u) & g.vmask) > half) m |= 1u << b;
      }
      return (int32_t)m;
    }
  }
  int32_t c = x;
  int32_t k = g.valid ? 1 : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {  // branch-free pair cancellation
    const int32_t c2 = __shfl_xor(c, o);
    const int32_t k2 = __shfl_xor(k, o);
    const uint32_t same = eq01(c, c2);
    const uint32_t keep = same | (1u - gt01(k2, k));  // c == c2 or k >= k2
    const int32_t diff = k - k2;
    const int32_t kn = same ? k + k2 : (diff < 0 ? -diff : diff);
    c = keep ? c : c2;
    k = kn;
  }
  if constexpr (W == 1) {
    return rfl32(c);
  } else {
    int64_t* s = g.red + g.ph * W;
    g.ph ^= 1;
    if (g.lane == 0) s[g.wv] = ((int64_t)k << 32) | (uint32_t)c;
    __syncthreads();
    int32_t cc = (int32_t)(uint32_t)s[0];
    int32_t kk = (int32_t)(s[0] >> 32);
    for (int w = 1; w < W; ++w) {
      const int32_t c2 = (int32_t)(uint32_t)s[w];
      const int32_t k2 = (int32_t)(s[w] >> 32);
      if (cc == c2) {
        kk += k2;
      } else if (kk >= k2) {
        kk -= k2;
      } else {
        cc = c2;
        kk = k2 - kk;
      }
    }
    return rfl32(cc);
  }
}

// Shared by FloodMin and KSet: slot 0 KAgreement (|{decisions of correct
// deciders}| <= k), slot 1 KValidity (every decision is an initial value).
// vote = mailbox.maxBy(_._2._2)._2._1 over a uniform mailbox Mc of (x, ts)
// messages (LastVoting.scala:132, ShortLastVoting.scala:43): the first maximal ts
// in Scala Map iteration order — insertion order (ascending pid) up to 4 entries,
// CHAMP order beyond, from per-lane CHAMP sort keys and a min-reduction. Only
// needed when the maximal-ts senders disagree on x.
template <int W>
PSG_DEV int32_t maxby_ts_x(Grp<W>& g, const int32_t* xs, const Mask<W>& Mc, int size, int32_t x, int32_t ts,
                           uint32_t myh, int tiebreak, const ChampTable<W>* CT = nullptr) {
  const bool inMc = mtest(Mc, g.pid);
  const int32_t maxts = g.max32(ts, inMc);
  const Mask<W> T = mand(Mc, g.ballot(ts == maxts));
  const int q0 = mfirst(T);
  const int32_t xq0 = g.bcast(x, xs, q0);
  int win = q0;
  const bool differ = many(mand(T, g.ballot(x != xq0)));
  if (differ && tiebreak == PSG_TIE_CHAMP && size > 4) {
    // payload depth of each candidate = longest 5-bit hash prefix shared with another entry.
    // h: an opaque copy of the lane's hash, so the fragment values derived from it are formed in
    // this (rare) block instead of hoisted out of the kernel's loops and held live
    uint32_t h = myh;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(h));
#endif
    int depth = 0;
    if (CT) {
      // per lane, level by level: the entries sharing this lane's first l+1 fragments are the
      // mailbox intersected with the table's fragment masks; depth = the levels where that set
      // still holds another entry (lane-parallel VALU + LDS instead of a scalar walk of the
      // mailbox with a hash per entry)
      Mask<W> S = Mc;
#pragma unroll
      for (int l = 0; l < 7; ++l) {
        const uint32_t f = (h >> (5 * l)) & 31u;
#pragma unroll
        for (int w = 0; w < W; ++w) S.w[w] &= CT->b[l][f][w];
        depth += mpopc(S) >= 2 ? 1 : 0;
      }
    } else {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        uint64_t m = Mc.w[w];
        while (m) {
          const int f = w * 64 + __builtin_ctzll(m);
          m &= m - 1;
          if (f != g.pid) depth = max(depth, champ_cpl(h, scala_improve((uint32_t)f)));
        }
      }
    }
    const bool inT = mtest(T, g.pid);
    const int64_t key = (int64_t)champ_key(h, depth);
    const int64_t kmin = g.min64(key, inT);
    win = mfirst(mand(T, g.ballot(key == kmin)));
  }
  return g.bcast(x, xs, win);
}

template <int W>
PSG_DEV void kagree_check(Grp<W>& g, Checks& ck, int c, int kk, const Mask<W>& full, bool decided, int32_t decision,
                          const X0Set<W>& X0, bool crashed, const int32_t* dstaged, bool alive = false,
                          Mask<W>* alive_out = nullptr) {
  // decided, decided by a correct process, decided a non-initial value: one exchange;
  // alive_out: the caller's next-round `act` ballot rides on the same exchange
  const bool pr[4] = {decided, decided && !crashed, decided && !X0.contains(decision), alive};
  Mask<W> m[4];
  g.template ballots<4>(pr, m);
  if (alive_out) *alive_out = m[3];
  Mask<W> Y = m[1];
  int distinct = 0;
  while (many(Y) && distinct <= kk) {
    const int32_t dv = g.bcast(decision, dstaged, mfirst(Y));
    Y = mandn(Y, g.ballot(decided && !crashed && decision == dv));
    ++distinct;
  }
  const bool valid = !many(m[2]);
  ck.record(fbit(distinct <= kk, 0) | fbit(valid, 1), meq(m[0], full), c, g.lane);
}


}  // namespace psg
