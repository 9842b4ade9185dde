// psg_spec_vm.hip — device interpreter for compiled Spec programs.
//
// A Formula tree (psync/formula/Formula.scala: ForAll / Exists / Comprehension /
// Cardinality over processes, V.exists over Int / Boolean, init(...) / old(...),
// Option isDefined / get) compiled by round_amd/formula.py into the stack
// bytecode of include/psg.h, evaluated after every round over a trace of the
// process states written by the round kernels (trace_put).
//
// One wave per instance. Values are per-lane int32 on an LDS stack; control is
// wave-uniform. Process quantifiers come in two forms chosen by the compiler:
// lane form (one lane per pid, 64 pids per pass, reduced with a ballot) for the
// outermost one, serial form (a uniform loop over pids, each lane carrying its
// own accumulator) when nested. V.exists over Int iterates the distinct values
// of the fields and expressions the variable is compared with, each -1/0/+1,
// plus Int.MinValue and Int.MaxValue: the body's truth value only changes at
// those values, so the finitization is exact. Quantifiers stop as soon as no
// further candidate can change any active lane's result.
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

constexpr int VM_STACK = 24;
constexpr int VM_VARS = 16;
constexpr int VM_FRAMES = 12;
constexpr int VM_VI_DEPTH = 2;  // nested V.exists over Int
constexpr int VM_VI_CAP = 1024; // distinct candidate bases per V.exists

enum { VM_ERR_STACK = 1, VM_ERR_FRAMES = 2, VM_ERR_VI = 4, VM_ERR_OP = 8 };

struct VmWave {
  int32_t stk[VM_STACK][64];
  int32_t var[VM_VARS][64];
  int32_t fr[VM_FRAMES][8];  // kind, var, body pc, end pc, idx, limit, vi depth, -
  uint64_t frl[VM_FRAMES];   // saved lane mask
  int32_t vi[VM_VI_DEPTH][VM_VI_CAP];
};

struct Vm {
  VmWave* w;
  const int32_t* code;
  const int32_t* cur;  // trace rows of check point c, c-1 (c = 0: c) and 0
  const int32_t* old;
  const int32_t* init;
  int n, r, lane;
  uint32_t err;

  PSG_DEV int32_t u(int32_t v) const { return __builtin_amdgcn_readfirstlane(v); }
  PSG_DEV uint64_t ballot(bool p) const { return __builtin_amdgcn_ballot_w64(p); }

  PSG_DEV int32_t field(int f, int tag, int32_t p) const {
    if (p < 0 || p >= n || f < 0 || f >= PSG_NFIELDS) return 0;
    const int32_t* t = tag == PSG_TAG_CUR ? cur : (tag == PSG_TAG_OLD ? old : init);
    return t[f * n + p];
  }

  // candidate k of a V.exists over Int with L bases: base(k/3) - 1 + k%3, then MIN, MAX
  PSG_DEV int32_t vi_cand(int depth, int k, int L) const {
    if (k < 3 * L) return (int32_t)((uint32_t)w->vi[depth][k / 3] + (uint32_t)(k % 3) - 1u);
    return k == 3 * L ? INT32_MIN : INT32_MAX;
  }

  // append the distinct values of `val` over the lanes in `m` to the base list
  PSG_DEV void vi_add(int depth, int& L, int32_t val, uint64_t m) {
    while (m) {
      const int q = __builtin_ctzll(m);
      const int32_t v = __builtin_amdgcn_readlane(val, q);
      m &= ~ballot(val == v);
      if (L < VM_VI_CAP) {
        if (lane == 0) w->vi[depth][L] = v;
        ++L;
      } else {
        err |= VM_ERR_VI;
        return;
      }
    }
  }

  // Evaluate the expression at pc (uniform context); returns its value.
  PSG_DEV int32_t eval(int pc) {
    int sp = 0, fp = 0, vid = 0;
    uint64_t lmask = ~0ull;  // lanes whose values matter (lane quantifier chunk)
#define PUSH(v)                                 \
  do {                                          \
    if (sp >= VM_STACK) { err |= VM_ERR_STACK; return 0; } \
    w->stk[sp][lane] = (v);                     \
    ++sp;                                       \
  } while (0)
#define POP() (w->stk[--sp][lane])
    while (true) {
      const int32_t word = u(code[pc]);
      const int op = word & 0xff;
      const int a = (word >> 8) & 0xff;
      const int b = word >> 16;
      ++pc;
      switch (op) {
        case PSG_OP_HALT: {
          const int32_t v = sp > 0 ? w->stk[sp - 1][lane] : 0;
          return u(v);
        }
        case PSG_OP_IMM: PUSH(b); break;
        case PSG_OP_IMM32: PUSH(u(code[pc])); ++pc; break;
        case PSG_OP_N: PUSH(n); break;
        case PSG_OP_R: PUSH(r); break;
        case PSG_OP_COORD: PUSH((r / 4) % n); break;
        case PSG_OP_VAR: PUSH(w->var[a][lane]); break;
        case PSG_OP_FIELD: {
          const int32_t p = POP();
          PUSH(field(a, b, p));
          break;
        }
        case PSG_OP_NOT: { const int32_t x = POP(); PUSH(x == 0 ? 1 : 0); break; }
        case PSG_OP_NEG: { const int32_t x = POP(); PUSH((int32_t)(0u - (uint32_t)x)); break; }
        case PSG_OP_ISDEF: { const int32_t x = POP(); PUSH(x != PSG_NONE32 ? 1 : 0); break; }
        case PSG_OP_BIND: { const int32_t x = POP(); w->var[a][lane] = x; break; }
        case PSG_OP_AND: case PSG_OP_OR: case PSG_OP_IMPL: case PSG_OP_EQ: case PSG_OP_NE: case PSG_OP_LT:
        case PSG_OP_LE: case PSG_OP_GT: case PSG_OP_GE: case PSG_OP_ADD: case PSG_OP_SUB: case PSG_OP_MUL:
        case PSG_OP_DIV: case PSG_OP_MOD: {
          const int32_t y = POP();
          const int32_t x = POP();
          int32_t z = 0;
          switch (op) {
            case PSG_OP_AND: z = (x != 0 && y != 0) ? 1 : 0; break;
            case PSG_OP_OR: z = (x != 0 || y != 0) ? 1 : 0; break;
            case PSG_OP_IMPL: z = (x == 0 || y != 0) ? 1 : 0; break;
            case PSG_OP_EQ: z = x == y; break;
            case PSG_OP_NE: z = x != y; break;
            case PSG_OP_LT: z = x < y; break;
            case PSG_OP_LE: z = x <= y; break;
            case PSG_OP_GT: z = x > y; break;
            case PSG_OP_GE: z = x >= y; break;
            case PSG_OP_ADD: z = (int32_t)((uint32_t)x + (uint32_t)y); break;
            case PSG_OP_SUB: z = (int32_t)((uint32_t)x - (uint32_t)y); break;
            case PSG_OP_MUL: z = (int32_t)((uint32_t)x * (uint32_t)y); break;
            case PSG_OP_DIV: z = (y == 0 || (x == INT32_MIN && y == -1)) ? (y == 0 ? 0 : x) : x / y; break;
            default: z = (y == 0 || y == -1) ? 0 : x % y; break;
          }
          PUSH(z);
          break;
        }
        case PSG_OP_QBEGIN: {
          if (fp >= VM_FRAMES) { err |= VM_ERR_FRAMES; return 0; }
          const int end = u(code[pc]);
          ++pc;
          int32_t* F = w->fr[fp];
          int limit = n, depth = 0;
          int32_t first = 0, acc = (a == PSG_Q_FORALL_P || a == PSG_Q_FORALL_PL) ? 1 : 0;
          if (a == PSG_Q_EXISTS_VI) {
            const int32_t desc = u(code[pc]);
            ++pc;
            const int nexpr = desc & 0xffff, nfs = (desc >> 16) & 0xffff;
            depth = vid++;
            if (depth >= VM_VI_DEPTH) { err |= VM_ERR_VI; return 0; }
            int L = 0;
            for (int e = 0; e < nexpr; ++e) {
              const int32_t v = POP();
              vi_add(depth, L, v, lmask);
            }
            for (int s = 0; s < nfs; ++s) {
              const int32_t fw = u(code[pc]);
              ++pc;
              for (int base = 0; base < n; base += 64) {
                const int p = base + lane;
                const int32_t v = p < n ? field(fw & 0xff, (fw >> 8) & 0xff, p) : 0;
                vi_add(depth, L, v, ballot(p < n));
              }
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
            limit = 3 * L + 2;
            first = vi_cand(depth, 0, L);
            F[5] = L;
          } else if (a == PSG_Q_EXISTS_VB) {
            limit = 2;
          }
          F[0] = a;
          F[1] = b;
          F[2] = pc;
          F[3] = end;
          F[4] = 0;
          if (a != PSG_Q_EXISTS_VI) F[5] = limit;
          F[6] = depth;
          w->frl[fp] = lmask;
          ++fp;
          if (a >= PSG_Q_FORALL_PL && a <= PSG_Q_COUNT_PL) {
            w->var[b][lane] = lane;
            lmask = ballot(lane < n);
          } else {
            w->var[b][lane] = first;
          }
          PUSH(acc);
          break;
        }
        case PSG_OP_QEND: {
          int32_t* F = w->fr[fp - 1];
          const int kind = u(F[0]), vb = u(F[1]), body = u(F[2]), end = u(F[3]);
          int idx = u(F[4]);
          const int32_t res = POP();
          int32_t acc = POP();
          bool more;
          if (kind >= PSG_Q_FORALL_PL && kind <= PSG_Q_COUNT_PL) {  // lane form: reduce this chunk
            const uint64_t t = ballot(res != 0) & lmask;
            if (kind == PSG_Q_FORALL_PL) acc = (acc != 0 && t == lmask) ? 1 : 0;
            else if (kind == PSG_Q_EXISTS_PL) acc = (acc != 0 || t != 0) ? 1 : 0;
            else acc += __builtin_popcountll(t);
            acc = u(acc);
            idx += 64;
            more = idx < n && !(kind == PSG_Q_FORALL_PL && acc == 0) && !(kind == PSG_Q_EXISTS_PL && acc != 0);
            if (more) {
              w->var[vb][lane] = idx + lane;
              lmask = ballot(idx + lane < n);
            }
          } else {  // serial form: per-lane accumulator
            if (kind == PSG_Q_FORALL_P) acc = (acc != 0 && res != 0) ? 1 : 0;
            else if (kind == PSG_Q_COUNT_P) acc += res != 0 ? 1 : 0;
            else acc = (acc != 0 || res != 0) ? 1 : 0;
            const uint64_t t = ballot(acc != 0) & lmask;
            ++idx;
            const int limit = u(F[5]);
            const int lim = kind == PSG_Q_EXISTS_VI ? 3 * limit + 2 : limit;
            more = idx < lim;
            if (kind == PSG_Q_FORALL_P && t == 0) more = false;
            if (kind != PSG_Q_FORALL_P && kind != PSG_Q_COUNT_P && t == lmask) more = false;
            if (more) {
              w->var[vb][lane] = kind == PSG_Q_EXISTS_VI ? vi_cand(u(F[6]), idx, limit) : idx;
            }
          }
          if (more) {
            F[4] = idx;
            PUSH(acc);
            pc = body;
          } else {
            --fp;
            lmask = w->frl[fp];
            if (kind == PSG_Q_EXISTS_VI) --vid;
            PUSH(acc);
            pc = end + 1;
          }
          break;
        }
        default:
          err |= VM_ERR_OP;
          return 0;
      }
    }
#undef PUSH
#undef POP
  }
};

__global__ void __launch_bounds__(64) spec_vm_kernel(VmArgs A) {
  __shared__ VmWave W;
  __shared__ BlockCounters bc;
  counters_init(&bc);
  __syncthreads();
  const int lane = threadIdx.x;
  const int n = A.n;
  const uint64_t rowsz = (uint64_t)PSG_NFIELDS * (uint64_t)n;
  uint32_t err = 0;
  for (uint64_t i = blockIdx.x; i < A.count; i += gridDim.x) {
    const int32_t* base = A.trace + i * (uint64_t)(A.R + 1) * rowsz;
    Vm vm;
    vm.w = &W;
    vm.code = A.code;
    vm.init = base;
    vm.n = n;
    vm.lane = lane;
    vm.err = 0;
    uint32_t failed = 0;
    int32_t ffv = PSG_NEVER;  // lane s: first failing check point of slot s
    int term = PSG_NEVER;
    for (int c = 0; c <= A.R; ++c) {
      vm.r = c;
      vm.cur = base + (uint64_t)c * rowsz;
      vm.old = base + (uint64_t)(c > 0 ? c - 1 : 0) * rowsz;
      for (int s = 0; s < A.n_slots; ++s) {
        const bool vacuous = c == 0 && (A.slot_flags[s] & PSG_SPEC_RELATIONAL);
        const bool ok = vacuous || vm.eval(A.slot_entry[s]) != 0;
        if (!ok && !((failed >> s) & 1u)) {
          failed |= 1u << s;
          if (lane == s) ffv = c;
        }
      }
      if (A.term_entry >= 0 && term == PSG_NEVER && vm.eval(A.term_entry) != 0) term = c;
    }
    err |= vm.err;
    if (A.out_inst) {
      uint8_t* o = reinterpret_cast<uint8_t*>(A.out_inst + i);
      if (lane < PSG_MAX_CHECKS) o[8 + lane] = (uint8_t)ffv;
      if (lane == 0) {
        o[8 + PSG_MAX_CHECKS] = (uint8_t)term;
        o[9 + PSG_MAX_CHECKS] = (uint8_t)A.n_slots;
      }
    }
    if (lane < A.n_slots && ((failed >> lane) & 1u)) atomicAdd(&bc.fail[lane], 1u);
    if (lane == 0) atomicAdd(&bc.hist[term == PSG_NEVER ? A.R + 1 : term], 1u);
  }
  if (err && lane == 0) atomicOr(A.err, (int32_t)err);
  __syncthreads();
  counters_flush(&bc, A.counters, A.n_slots, A.R);
}

hipError_t launch_spec_vm(const VmArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(spec_vm_kernel, dim3(grid), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace psg
