// psg_population.hip — device-resident adversary-search populations
// (psg_population_fresh / psg_population_next, include/psg.h).
//
// The search (round_amd/adversary.py) evaluates populations
// of explicit HO schedules; generating and mutating them on the host made the
// host the bottleneck (10 KB of HO sets per n=64, R=20 schedule over PCIe, numpy
// bit twiddling). Here a generation is four elementwise kernels over HBM:
//   links  — one thread per HO set (instance i, round k, process p): a fresh set
//            (each link present w.p. keep/256: 8 binary digits, x = r | x for a
//            1 digit, r & x for a 0 digit, fresh Philox words r) or a copy of the
//            parent's set; bits >= n cleared;
//   flip   — one thread per (instance, flip): a mutant toggles `flips` random
//            links (64-bit atomic xor: two flips may share a word);
//   repair — one thread per HO set: self bit, then random senders are added
//            until |HO(p)| >= min_size (the Specs' safety predicate, e.g. BenOr's
//            |HO(p)| > n/2, example/BenOr.scala:92);
//   init   — one thread per process: copy, redraw w.p. redraw/256, or fresh.
// Every draw is Philox4x32-10 keyed by the population seed with counter
// (slot, generation, k*n + p, tag | s), so a population is a pure function of its
// parameters (tests recompute them on the host).
#include <algorithm>

#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

constexpr uint32_t TAG_LINKS = 0xA000u << 16, TAG_REPAIR = 0xB000u << 16, TAG_FLIP = 0xC000u << 16,
                   TAG_INIT = 0xD000u << 16;

PSG_DEV U4 pop_draw(const PopArgs& a, uint64_t slot, uint32_t c2, uint32_t c3) {
  return philox10((uint32_t)slot, a.gen, c2, c3, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
}

PSG_DEV uint64_t full_word(int n, int w) {
  const int b = n - 64 * w;
  return b >= 64 ? ~0ull : (b <= 0 ? 0ull : ((1ull << b) - 1ull));
}

__global__ void __launch_bounds__(256) pop_links_kernel(PopArgs a) {
  const uint64_t sets = a.count * (uint64_t)a.R * (uint64_t)a.n;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < sets; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / ((uint64_t)a.R * a.n);
    const uint32_t kp = (uint32_t)(e - i * (uint64_t)a.R * a.n);  // k * n + p
    const int op = a.op ? a.op[i] : 2;
    uint64_t* dst = a.ho + e * a.W;
    if (op == 2) {
      const uint32_t q = a.keep[i & 3u];  // keep/256, 8 binary digits
      for (int w = 0; w < a.W; ++w) {
        uint64_t x;
        if (q >= 256u) {
          x = ~0ull;
        } else {
          x = 0;
          for (uint32_t j = 0; j < 8; j += 2) {  // digits j, j+1 from one call
            const U4 o = pop_draw(a, i, kp, TAG_LINKS | (uint32_t)(w * 4 + j / 2));
            const uint64_t r0 = (uint64_t)o.x | ((uint64_t)o.y << 32);
            const uint64_t r1 = (uint64_t)o.z | ((uint64_t)o.w << 32);
            x = ((q >> j) & 1u) ? (r0 | x) : (r0 & x);
            x = ((q >> (j + 1)) & 1u) ? (r1 | x) : (r1 & x);
          }
        }
        dst[w] = x & full_word(a.n, w);
      }
    } else {
      const uint64_t* src = a.src + ((uint64_t)a.parent[i] * a.R * a.n + kp) * a.W;
      for (int w = 0; w < a.W; ++w) dst[w] = src[w] & full_word(a.n, w);
    }
  }
}

__global__ void __launch_bounds__(256) pop_flip_kernel(PopArgs a) {
  const uint64_t total = a.count * (uint64_t)a.flips;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / a.flips;
    const uint32_t f = (uint32_t)(e - i * a.flips);
    if (a.op[i] != 1) continue;
    const U4 o = pop_draw(a, i, f, TAG_FLIP);
    const uint32_t k = mulhi32(o.x, (uint32_t)a.R);
    const uint32_t p = mulhi32(o.y, (uint32_t)a.n);
    uint32_t q = mulhi32(o.z, (uint32_t)a.n);
    if (a.self_bit && q == p) q = (q + 1u) % (uint32_t)a.n;
    unsigned long long* word =
        reinterpret_cast<unsigned long long*>(a.ho + ((i * a.R + k) * (uint64_t)a.n + p) * a.W + (q >> 6));
    atomicXor(word, 1ull << (q & 63u));
  }
}

__global__ void __launch_bounds__(256) pop_repair_kernel(PopArgs a) {
  const uint64_t sets = a.count * (uint64_t)a.R * (uint64_t)a.n;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < sets; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / ((uint64_t)a.R * a.n);
    const uint32_t kp = (uint32_t)(e - i * (uint64_t)a.R * a.n);
    const uint32_t p = kp % (uint32_t)a.n;
    uint64_t* s = a.ho + e * a.W;
    if (a.self_bit) s[p >> 6] |= 1ull << (p & 63u);
    if (a.min_size <= 0) continue;
    auto size = [&]() {
      int c = 0;
      for (int w = 0; w < a.W; ++w) c += __popcll(s[w]);
      return c;
    };
    uint32_t t = 0;
    while (size() < a.min_size && t < 64) {  // add random senders (each w.p. 1/2) until large enough
      for (int w = 0; w < a.W; ++w) {
        const U4 o = pop_draw(a, i, kp, TAG_REPAIR | (t * 8u + (uint32_t)w));
        s[w] |= ((uint64_t)o.x | ((uint64_t)o.y << 32)) & full_word(a.n, w);
      }
      ++t;
    }
    if (size() < a.min_size)
      for (int w = 0; w < a.W; ++w) s[w] = full_word(a.n, w);
  }
}

__global__ void __launch_bounds__(256) pop_init_kernel(PopArgs a) {
  const uint64_t cells = a.count * (uint64_t)a.n;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < cells; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / a.n;
    const uint32_t p = (uint32_t)(e - i * a.n);
    const int op = a.op ? a.op[i] : 2;
    const U4 o = pop_draw(a, i, p, TAG_INIT);
    const int32_t fresh = a.benor ? (int32_t)(o.y & 1u) : 1 + (int32_t)mulhi32(o.y, (uint32_t)a.V);
    int32_t v = fresh;
    if (op != 2) {
      v = a.src_init[(uint64_t)a.parent[i] * a.n + p];
      if (op == 1 && (o.x >> 24) < a.redraw) v = fresh;
    }
    a.init[e] = v;
  }
}

hipError_t launch_population(const PopArgs& a, hipStream_t s) {
  const uint64_t sets = a.count * (uint64_t)a.R * (uint64_t)a.n;
  auto grid = [](uint64_t work) { return (int)std::min<uint64_t>((work + 255) / 256, 16384); };
  if (sets == 0) return hipSuccess;
  hipLaunchKernelGGL(pop_links_kernel, dim3(grid(sets)), dim3(256), 0, s, a);
  if (a.op && a.flips) hipLaunchKernelGGL(pop_flip_kernel, dim3(grid(a.count * a.flips)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pop_repair_kernel, dim3(grid(sets)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(pop_init_kernel, dim3(grid(a.count * (uint64_t)a.n)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace psg
