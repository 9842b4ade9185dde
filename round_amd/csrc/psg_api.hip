// psg_api.hip — C ABI of include/psg.h: context, device buffers, launches.
//
// Replaces, for simulation, the reference's Runtime + InstanceHandler round
// loop (psync/runtime/Runtime.scala:60-93, psync/runtime/InstanceHandler.scala:164-258):
// one psg_run_batch call starts every instance of a range and runs all its
// rounds inside one kernel launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/psg.h"
#include "psg_device.hpp"
#include "psg_kernels.hpp"

namespace psg {

// Seeded synthetic initial values (the ConsensusIO.initialValue of every process).
__global__ void gen_init_kernel(uint64_t inst_begin, uint64_t count, int n, int alg, int V, uint64_t seed,
                                int32_t* out) {
  const uint64_t total = count * (uint64_t)n;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = e / (uint64_t)n;
    const int p = (int)(e - i * (uint64_t)n);
    const uint64_t w = rword(seed, inst_begin + i, ROUND_INIT, (uint32_t)p, 0);
    out[e] = alg == PSG_ALG_BENOR ? (int32_t)((uint32_t)w & 1u) : 1 + (int32_t)mulhi32((uint32_t)w, (uint32_t)V);
  }
}

hipError_t launch_gen_init(uint64_t inst_begin, uint64_t count, int n, int alg, int V, uint64_t seed, int32_t* out,
                           hipStream_t s) {
  const uint64_t total = count * (uint64_t)n;
  const int grid = (int)std::min<uint64_t>((total + 255) / 256, 8192);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_init_kernel, dim3(grid), dim3(256), 0, s, inst_begin, count, n, alg, V, seed, out);
  return hipGetLastError();
}

}  // namespace psg

using namespace psg;

struct psg_ctx {
  psg_config cfg;
  int W = 1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  uint64_t cap = 0;
  int32_t* d_init = nullptr;
  double* d_init_f64 = nullptr;  // EpsilonConsensus: staged host Double inputs
  bool init_f64_host = false;    // false: seeded Doubles generated inside the round kernel
  double* d_dec_f64 = nullptr;
  double* d_rec_f64 = nullptr;   // fetch path: [k][n][2] (decision, final x)
  int32_t* d_trace = nullptr;    // psg_run_batch_spec: state trace of one chunk
  uint64_t trace_cap = 0;        // instances the trace buffer holds
  unsigned long long* d_vm_counters = nullptr;
  int32_t* d_vm_err = nullptr;
  int32_t* d_prog = nullptr;     // code | slot_entry | slot_flags
  size_t prog_cap = 0;
  std::string module_path;       // native Spec code object currently loaded
  hipModule_t module = nullptr;
  hipFunction_t native_fn = nullptr;
  hipFunction_t fused_fn = nullptr, fused_x_fn = nullptr;  // fused Spec module: round kernel + Spec
  int32_t module_alg = 0;        // the module's psg_spec_alg (0: not recorded)
  bool staged = false;
  bool staged_host = false;      // the staged rows came from the host (else seeded values)
  uint64_t staged_begin = 0, staged_count = 0;
  // explicit schedule (psg_load_schedule)
  uint64_t* d_ho = nullptr;
  int32_t* d_crash = nullptr;
  uint64_t ho_cap = 0;  // instances d_ho / d_crash hold
  bool ho_loaded = false, ho_has_crash = false;
  uint64_t ho_begin = 0, ho_count = 0;
  // search populations (psg_population_*): second buffers of the HO sets / inputs
  uint64_t* d_ho2 = nullptr;
  int32_t* d_init2 = nullptr;
  uint32_t* d_parent = nullptr;
  uint8_t* d_op = nullptr;
  uint64_t pop_cap = 0;
  int32_t* d_dec = nullptr;
  uint8_t* d_dround = nullptr;
  psg_instance_summary* d_inst = nullptr;
  unsigned long long* d_counters = nullptr;
  uint64_t* d_ids = nullptr;
  psg_process_record* d_rec = nullptr;
  uint64_t fetch_cap = 0;
  uint64_t last_count = 0;
  int grid_max = 0;  // resident blocks for the algorithm's kernel
  // packed KSet (n > 64): state handed from the general-round kernel to the uniform-t tail
  // kernel, per batch row a header word, 64 lane words and n decisions (psg_kset.hip)
  uint64_t* d_hand = nullptr;
  std::string err;
  // multi-device context (cfg.n_devices > 0): one single-device context per listed
  // device; every call splits its range into contiguous slices, one per device
  std::vector<psg_ctx*> subs;
};

static thread_local std::string g_create_err;

static int n_checks(int alg) {
  switch (alg) {
    case PSG_ALG_OTR: return 8;
    case PSG_ALG_LAST_VOTING: return 7;
    case PSG_ALG_BENOR: return 5;
    case PSG_ALG_FLOODMIN: return 2;
    case PSG_ALG_KSET: return 2;
    case PSG_ALG_OTR2: return 8;
    case PSG_ALG_SLV: return 2;
    case PSG_ALG_KSET_ES: return 2;
    case PSG_ALG_EPSILON: return 3;
  }
  return 0;
}

static const char* const k_names_otr[] = {"Safety", "Invariant0", "Invariant1", "Invariant2",
                                          "Agreement", "Validity", "Integrity", "Irrevocability"};
static const char* const k_names_lv[] = {"Safety", "Invariant0", "Invariant1", "Agreement",
                                         "Validity", "Integrity", "Irrevocability"};
static const char* const k_names_benor[] = {"Safety", "Invariant0", "Agreement", "Irrevocability", "SafetyPredicate"};
static const char* const k_names_k[] = {"KAgreement", "KValidity"};
static const char* const k_names_eps[] = {"EpsAgreement", "EpsValidity", "SafetyPredicate"};

static int fail(psg_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

static int hip_fail(psg_ctx* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? PSG_ENOMEM : PSG_EIO, m);
}

#define HIPCHK(ctx, call)                                  \
  do {                                                     \
    hipError_t e_ = (call);                                \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, #call); \
  } while (0)

// Profiling builds (-DPSG_PHASE_TIMERS=1): per-phase cycles, shader clock, wave lifetimes.
static void print_timers(const unsigned long long* host) {
  if (!PSG_PHASE_TIMERS) return;
  const unsigned long long* t = host + C_TIMER;
  const unsigned long long waves = t[T_WAVES], t0 = ~t[T_RT_MIN], span = t[T_RT_MAX] - ~t[T_RT_MIN];
  unsigned long long cyc = 0;
  std::fprintf(stderr, "psg phase cycles (kernel's own phase map):");
  for (int j = 0; j < NTIMERS; ++j) {
    std::fprintf(stderr, " t%d %llu", j, t[j]);
    cyc += t[j];
  }
  std::fprintf(stderr, "\n");
  std::fprintf(stderr, "psg wave lifetime: waves %llu, sum %llu rt ticks (100 MHz), span %llu ticks, mean/span %.3f, "
               "shader clock %.3f GHz\n", waves, t[T_RT_SUM], span,
               waves ? (double)t[T_RT_SUM] / waves / (double)span : 0.0,
               t[T_RT_SUM] ? 0.1 * cyc / (double)t[T_RT_SUM] : 0.0);
  // deciles of wave start and end times, as fractions of the span
  const size_t m = std::min<unsigned long long>(waves, NSTAMP_WAVES);
  std::vector<double> st(m), en(m);
  for (size_t w = 0; w < m; ++w) {
    st[w] = (double)(t[T_STAMPS + 2 * w] - t0) / span;
    en[w] = (double)(t[T_STAMPS + 1 + 2 * w] - t0) / span;
  }
  std::sort(st.begin(), st.end());
  std::sort(en.begin(), en.end());
  if (!m) return;
  std::fprintf(stderr, "psg wave start deciles:");
  for (int d = 0; d <= 10; ++d) std::fprintf(stderr, " %.3f", st[std::min(m - 1, d * m / 10)]);
  std::fprintf(stderr, "\npsg wave end deciles:  ");
  for (int d = 0; d <= 10; ++d) std::fprintf(stderr, " %.3f", en[std::min(m - 1, d * m / 10)]);
  std::fprintf(stderr, "\n");
}

static hipError_t launch_alg(const psg_ctx* c, const KArgs& a, int grid) {
  switch (c->cfg.alg) {
    case PSG_ALG_OTR: return launch_otr(a, c->W, grid, c->stream);
    case PSG_ALG_LAST_VOTING: return launch_lv(a, c->W, grid, c->stream);
    case PSG_ALG_FLOODMIN: return launch_floodmin(a, c->W, grid, c->stream);
    case PSG_ALG_KSET: return launch_kset(a, c->W, grid, c->stream);
    case PSG_ALG_BENOR: return launch_benor(a, c->W, grid, c->stream);
    case PSG_ALG_OTR2: return launch_otr2(a, c->W, grid, c->stream);
    case PSG_ALG_SLV: return launch_slv(a, c->W, grid, c->stream);
    case PSG_ALG_KSET_ES: return launch_kset_es(a, c->W, grid, c->stream);
    case PSG_ALG_EPSILON: return launch_epsilon(a, c->W, grid, c->stream);
  }
  return hipErrorInvalidValue;
}

static const void* kernel_ptr(int alg, int W) {
  switch (alg) {
    case PSG_ALG_OTR: return otr_kernel_ptr(W);
    case PSG_ALG_LAST_VOTING: return lv_kernel_ptr(W);
    case PSG_ALG_FLOODMIN: return floodmin_kernel_ptr(W);
    case PSG_ALG_KSET: return kset_kernel_ptr(W);
    case PSG_ALG_BENOR: return benor_kernel_ptr(W);
    case PSG_ALG_OTR2: return otr2_kernel_ptr(W);
    case PSG_ALG_SLV: return slv_kernel_ptr(W);
    case PSG_ALG_KSET_ES: return kset_es_kernel_ptr(W);
    case PSG_ALG_EPSILON: return epsilon_kernel_ptr(W);
  }
  return nullptr;
}

static KArgs make_args(const psg_ctx* c) {
  KArgs a;
  std::memset(&a, 0, sizeof(a));
  const psg_config& f = c->cfg;
  a.seed = f.seed;
  a.n = f.n;
  a.R = f.rounds;
  a.V = f.value_range;
  a.param = f.param;
  a.param2 = f.param2;
  a.real_param = f.real_param;
  a.variant = f.variant;
  a.tiebreak = f.tiebreak;
  a.drop_log2 = f.sched.drop_log2;
  a.good_p32 = f.sched.good_p32;
  a.good_min = f.sched.good_min;
  // at most 0 crashes: f = mulhi32(w, fmax + 1) = 0 for every instance, so nobody crashes — the
  // kernels skip the instance's crash draws and the per-round crash sets (the same schedule)
  a.crash_fmax = f.sched.crash_fmax == 0 ? -1 : f.sched.crash_fmax;
  a.ho_min = f.sched.ho_min;
  a.self_bit = f.sched.self_bit;
  a.counters = c->d_counters;
  if (c->d_hand) {
    a.hand_hdr = c->d_hand;
    a.hand_meta = c->d_hand + c->cap;
    a.hand_dec = reinterpret_cast<int32_t*>(c->d_hand + c->cap * 65);
  }
  if (c->ho_loaded) {
    a.ho_in = c->d_ho;
    a.crash_in = c->ho_has_crash ? c->d_crash : nullptr;
    a.ho_base = c->ho_begin;
  }
  return a;
}

// Instances [begin, begin+count) must lie inside a loaded explicit schedule.
static int check_sched_range(psg_ctx* c, uint64_t begin, uint64_t count) {
  if (!c->ho_loaded || count == 0) return PSG_OK;
  if (begin < c->ho_begin || begin - c->ho_begin > c->ho_count || count > c->ho_count - (begin - c->ho_begin))
    return fail(c, PSG_ERANGE, "instances outside the loaded explicit schedule");
  return PSG_OK;
}

static int groups_per_block(int W) { return W == 1 ? 4 : 1; }

static int run_kernel(psg_ctx* c, KArgs& a, uint64_t count, psg_summary* out, bool timed) {
  const int G = groups_per_block(c->W);
  uint64_t want = (count + G - 1) / G;
  int grid = (int)std::min<uint64_t>(want, (uint64_t)c->grid_max);
  if (grid < 1) grid = 1;
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, sizeof(unsigned long long) * NCOUNTERS_ALLOC, c->stream));
  if (timed) HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, launch_alg(c, a, grid));
  if (timed) HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  unsigned long long host[NCOUNTERS_ALLOC];
  HIPCHK(c, hipMemcpyAsync(host, c->d_counters, sizeof(host), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (PSG_PHASE_TIMERS && std::getenv("PSG_PHASE_TIMERS")) print_timers(host);
  if (out) {
    std::memset(out, 0, sizeof(*out));
    out->instances = (int64_t)count;
    out->process_rounds = (int64_t)count * c->cfg.n * c->cfg.rounds;
    out->active_process_rounds = (int64_t)host[C_ACTIVE];
    out->live_instance_rounds = (int64_t)host[C_LIVE];
    for (int i = 0; i < PSG_MAX_CHECKS; ++i) out->fail_count[i] = (int64_t)host[C_FAIL + i];
    out->decided_processes = (int64_t)host[C_DECIDED];
    out->digest = (int64_t)host[C_DIGEST];
    for (int i = 0; i < c->cfg.rounds + 2; ++i) out->term_hist[i] = (int64_t)host[C_HIST + i];
    if (timed) {
      float ms = 0.f;
      HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
      out->kernel_ns = (int64_t)((double)ms * 1e6);
    }
  }
  return PSG_OK;
}

// psg_selftest_bitset: LongBitSet's operations (LongBitSet.scala:7-23) on Mask<W>, one lane
template <int W>
__global__ void bitset_selftest_kernel(const int32_t* ops, int n_ops, int32_t* out, int n_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Mask<W> m = mzero<W>();
  int o = 0;
  for (int i = 0; i < n_ops; ++i) {
    // index mod 64W on the signed value (Java's shift masks to mod 64 for W = 1; -1 -> 64W - 1)
    const int op = ops[2 * i], pos = ((ops[2 * i + 1] % (64 * W)) + 64 * W) % (64 * W);
    switch (op) {
      case 0: m = mzero<W>(); break;
      case 1: m = mfull<W>(64 * W); break;
      case 2: mset(m, pos); break;
      case 3: mclear(m, pos); break;
      case 4:
        if (mtest(m, pos)) mclear(m, pos);
        else mset(m, pos);
        break;
      case 5: if (o < n_out) out[o++] = mtest(m, pos) ? 1 : 0; break;
      case 6: if (o < n_out) out[o++] = mpopc(m); break;
      default: break;
    }
  }
}

extern "C" {

int psg_config_default(psg_config* cfg, int32_t alg, int32_t n) {
  if (!cfg) return PSG_EINVAL;
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->abi_version = PSG_ABI_VERSION;
  cfg->alg = alg;
  cfg->n = n;
  cfg->rounds = 20;
  cfg->seed = 1;
  cfg->value_range = 4;
  cfg->param = 0;
  cfg->tiebreak = PSG_TIE_CHAMP;
  cfg->batch_capacity = 1u << 20;
  cfg->sched.drop_log2 = 3;
  cfg->sched.good_p32 = 1u << 30;
  cfg->sched.good_min = -1;
  cfg->sched.crash_fmax = -1;
  cfg->sched.ho_min = -1;
  cfg->sched.self_bit = 1;
  switch (alg) {
    case PSG_ALG_OTR: cfg->param = 2; break;  // afterDecision (Otr.scala:89)
    case PSG_ALG_LAST_VOTING:
      cfg->value_range = (1 << 15) - 1;
      cfg->sched.drop_log2 = 4;
      cfg->sched.good_p32 = 0;
      cfg->sched.crash_fmax = (n - 1) / 2;
      break;
    case PSG_ALG_FLOODMIN:
      cfg->param = 2;
      cfg->rounds = 4;
      cfg->value_range = 1000000;
      cfg->sched.drop_log2 = 0;
      cfg->sched.good_p32 = 0;
      cfg->sched.crash_fmax = 2;
      break;
    case PSG_ALG_KSET:
      cfg->param = 2;
      cfg->rounds = 16;
      cfg->value_range = 1000000;
      cfg->sched.drop_log2 = 0;
      cfg->sched.good_p32 = 0;
      cfg->sched.crash_fmax = 1;
      break;
    case PSG_ALG_BENOR:
      cfg->rounds = 64;
      cfg->value_range = 2;
      cfg->sched.drop_log2 = 2;
      cfg->sched.good_p32 = 0;
      cfg->sched.ho_min = n / 2;
      break;
    case PSG_ALG_OTR2: cfg->param = 2; break;  // afterDecision (Otr2.scala:69)
    case PSG_ALG_SLV:
      cfg->rounds = 30;
      cfg->value_range = (1 << 15) - 1;
      cfg->sched.drop_log2 = 4;
      cfg->sched.good_p32 = 0;
      cfg->sched.crash_fmax = (n - 1) / 2;
      break;
    case PSG_ALG_EPSILON:  // f = 1, epsilon = 0.1 (Epsilon.scala:83-89)
      cfg->param = 1;
      cfg->real_param = 0.1;
      cfg->rounds = 12;
      cfg->sched.drop_log2 = 4;
      cfg->sched.good_p32 = 0;
      cfg->sched.ho_min = n - 2;  // |HO(p)| >= n - f
      break;
    case PSG_ALG_KSET_ES:  // t = 2, k = 2 (KSetEarlyStopping.scala:63-67)
      cfg->param = 2;
      cfg->param2 = 2;
      cfg->rounds = 3;
      cfg->value_range = 1000000;
      cfg->sched.drop_log2 = 0;
      cfg->sched.good_p32 = 0;
      cfg->sched.crash_fmax = 2;
      break;
    default: return PSG_EINVAL;
  }
  return PSG_OK;
}

int psg_check_count(int32_t alg) { return n_checks(alg); }

const char* psg_check_name(int32_t alg, int32_t slot) {
  if (slot < 0 || slot >= n_checks(alg)) return nullptr;
  switch (alg) {
    case PSG_ALG_OTR:
    case PSG_ALG_OTR2: return k_names_otr[slot];
    case PSG_ALG_LAST_VOTING: return k_names_lv[slot];
    case PSG_ALG_BENOR: return k_names_benor[slot];
    case PSG_ALG_EPSILON: return k_names_eps[slot];
    default: return k_names_k[slot];
  }
}

int psg_alg_from_class(const char* name) {
  if (!name) return PSG_EINVAL;
  static const struct { const char* n; int id; } tab[] = {
      {"example.OTR", PSG_ALG_OTR}, {"example.LastVoting", PSG_ALG_LAST_VOTING},
      {"example.FloodMin", PSG_ALG_FLOODMIN}, {"example.KSetAgreement", PSG_ALG_KSET},
      {"example.BenOr", PSG_ALG_BENOR}, {"example.OTR2", PSG_ALG_OTR2},
      {"example.ShortLastVoting", PSG_ALG_SLV}, {"example.KSetEarlyStopping", PSG_ALG_KSET_ES},
      {"example.EpsilonConsensus", PSG_ALG_EPSILON}};
  for (auto& t : tab)
    if (std::strcmp(t.n, name) == 0) return t.id;
  return PSG_EINVAL;
}

const char* psg_create_error(void) { return g_create_err.c_str(); }

int psg_selftest_map_head(int32_t device, const uint64_t* sets, int32_t count, int32_t tiebreak, int32_t* out_first) {
  if (!sets || !out_first || count < 0) return PSG_EINVAL;
  if (tiebreak != PSG_TIE_CHAMP && tiebreak != PSG_TIE_MIN_PID) return PSG_EINVAL;
  if (count == 0) return PSG_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return PSG_ENODEV;
  if (hipSetDevice(device) != hipSuccess) return PSG_ENODEV;
  uint64_t* d_sets = nullptr;
  int32_t* d_out = nullptr;
  int rc = PSG_OK;
  if (hipMalloc(&d_sets, sizeof(uint64_t) * count) != hipSuccess ||
      hipMalloc(&d_out, sizeof(int32_t) * count) != hipSuccess) {
    rc = PSG_ENOMEM;
  } else if (hipMemcpy(d_sets, sets, sizeof(uint64_t) * count, hipMemcpyHostToDevice) != hipSuccess ||
             launch_champ_selftest(d_sets, count, tiebreak, d_out, nullptr) != hipSuccess ||
             hipMemcpy(out_first, d_out, sizeof(int32_t) * count, hipMemcpyDeviceToHost) != hipSuccess) {
    rc = PSG_EIO;
  }
  if (d_sets) (void)hipFree(d_sets);
  if (d_out) (void)hipFree(d_out);
  return rc;
}

int psg_selftest_bitset(int32_t device, int32_t W, const int32_t* ops, int32_t n_ops, int32_t* out, int32_t n_out) {
  if (!ops || !out || n_ops < 0 || n_out < 0 || W < 1 || W > 4) return PSG_EINVAL;
  if (n_ops == 0) return PSG_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return PSG_ENODEV;
  if (hipSetDevice(device) != hipSuccess) return PSG_ENODEV;
  int32_t *d_ops = nullptr, *d_out = nullptr;
  int rc = PSG_OK;
  const size_t ob = sizeof(int32_t) * (n_out > 0 ? n_out : 1);
  if (hipMalloc(&d_ops, sizeof(int32_t) * 2 * (size_t)n_ops) != hipSuccess || hipMalloc(&d_out, ob) != hipSuccess) {
    rc = PSG_ENOMEM;
  } else if (hipMemcpy(d_ops, ops, sizeof(int32_t) * 2 * (size_t)n_ops, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemset(d_out, 0xFF, ob) != hipSuccess) {
    rc = PSG_EIO;
  } else {
    switch (W) {
      case 1: hipLaunchKernelGGL(bitset_selftest_kernel<1>, dim3(1), dim3(64), 0, nullptr, d_ops, n_ops, d_out, n_out); break;
      case 2: hipLaunchKernelGGL(bitset_selftest_kernel<2>, dim3(1), dim3(64), 0, nullptr, d_ops, n_ops, d_out, n_out); break;
      case 3: hipLaunchKernelGGL(bitset_selftest_kernel<3>, dim3(1), dim3(64), 0, nullptr, d_ops, n_ops, d_out, n_out); break;
      default: hipLaunchKernelGGL(bitset_selftest_kernel<4>, dim3(1), dim3(64), 0, nullptr, d_ops, n_ops, d_out, n_out); break;
    }
    if (hipGetLastError() != hipSuccess ||
        (n_out > 0 && hipMemcpy(out, d_out, sizeof(int32_t) * n_out, hipMemcpyDeviceToHost) != hipSuccess))
      rc = PSG_EIO;
  }
  if (d_ops) (void)hipFree(d_ops);
  if (d_out) (void)hipFree(d_out);
  return rc;
}

static int validate(const psg_config* cfg, std::string& m) {
  if (!cfg) { m = "null config"; return PSG_EINVAL; }
  if (cfg->abi_version != PSG_ABI_VERSION) { m = "ABI version mismatch"; return PSG_EINVAL; }
  if (cfg->alg < PSG_ALG_OTR || cfg->alg > PSG_ALG_EPSILON) { m = "unknown algorithm"; return PSG_EINVAL; }
  if (cfg->n < 1 || cfg->n > PSG_MAX_N) { m = "n out of range 1..256"; return PSG_EINVAL; }
  if (cfg->rounds < 1 || cfg->rounds > PSG_MAX_ROUNDS) { m = "rounds out of range 1..250"; return PSG_EINVAL; }
  if (cfg->alg != PSG_ALG_BENOR && cfg->alg != PSG_ALG_EPSILON && cfg->value_range < 1) {
    m = "value_range must be >= 1";
    return PSG_EINVAL;
  }
  if (cfg->alg == PSG_ALG_EPSILON && (cfg->param < 1 || !(cfg->real_param > 0.0))) {
    m = "EpsilonConsensus needs f >= 1 and epsilon > 0";
    return PSG_EINVAL;
  }
  if (cfg->alg == PSG_ALG_KSET && cfg->param < 1) { m = "KSetAgreement needs k >= 1"; return PSG_EINVAL; }
  if (cfg->alg == PSG_ALG_FLOODMIN && cfg->param < 0) { m = "FloodMin needs f >= 0"; return PSG_EINVAL; }
  if ((cfg->alg == PSG_ALG_OTR || cfg->alg == PSG_ALG_OTR2) && cfg->param < 1) {
    m = "OTR needs afterDecision >= 1";
    return PSG_EINVAL;
  }
  if (cfg->alg == PSG_ALG_KSET_ES && (cfg->param < 0 || cfg->param2 < 1)) {
    m = "KSetEarlyStopping needs t >= 0 and k >= 1";
    return PSG_EINVAL;
  }
  if (cfg->tiebreak != PSG_TIE_CHAMP && cfg->tiebreak != PSG_TIE_MIN_PID) { m = "bad tiebreak"; return PSG_EINVAL; }
  if (cfg->sched.drop_log2 > 16) { m = "drop_log2 > 16"; return PSG_EINVAL; }
  if (cfg->batch_capacity < 1) { m = "batch_capacity must be >= 1"; return PSG_EINVAL; }
  if (cfg->n_devices < 0 || cfg->n_devices > PSG_MAX_DEVICES) { m = "n_devices out of range 0..16"; return PSG_EINVAL; }
  return PSG_OK;
}

// ---------------------------------------------------------------- multi-device contexts
// psg_config.n_devices > 0: the context owns one single-device context per listed
// device. A call over instances [begin, begin+count) gives device d the contiguous
// slice [begin + count*d/nd, begin + count*(d+1)/nd); the devices run concurrently,
// one host thread each, and their summaries are summed (kernel_ns: the maximum).
// Results equal a single-device run bit for bit (every draw is keyed on the global
// instance id). Under a loaded explicit schedule a multi-device run covers exactly
// the loaded range (its slices are the schedule's slices).
extern "C++" {
static void split(uint64_t count, size_t nd, size_t d, uint64_t& off, uint64_t& m) {
  off = count * d / nd;
  m = count * (d + 1) / nd - off;
}

template <class F>
static int par_subs(psg_ctx* c, F&& f) {
  const size_t nd = c->subs.size();
  std::vector<int> rc(nd, PSG_OK);
  std::vector<std::thread> th;
  try {
    th.reserve(nd);
    for (size_t d = 1; d < nd; ++d) th.emplace_back([&rc, &f, d] { rc[d] = f(d); });
  } catch (...) {
    for (auto& t : th) t.join();
    return fail(c, PSG_EIO, "could not start a host thread per device");
  }
  rc[0] = f(0);
  for (auto& t : th) t.join();
  for (size_t d = 0; d < nd; ++d)
    if (rc[d]) return fail(c, rc[d], "device " + std::to_string(c->cfg.devices[d]) + ": " + c->subs[d]->err);
  return PSG_OK;
}

static void summary_add(psg_summary& acc, const psg_summary& p) {
  acc.instances += p.instances;
  acc.process_rounds += p.process_rounds;
  acc.active_process_rounds += p.active_process_rounds;
  acc.live_instance_rounds += p.live_instance_rounds;
  for (int i = 0; i < PSG_MAX_CHECKS; ++i) acc.fail_count[i] += p.fail_count[i];
  acc.decided_processes += p.decided_processes;
  acc.digest = (int64_t)((uint64_t)acc.digest + (uint64_t)p.digest);
  for (int i = 0; i < PSG_MAX_ROUNDS + 2; ++i) acc.term_hist[i] += p.term_hist[i];
  acc.kernel_ns = std::max(acc.kernel_ns, p.kernel_ns);
}
}  // extern "C++"

static int create_multi(psg_ctx** out, const psg_config* cfg) {
  psg_ctx* c = new (std::nothrow) psg_ctx();
  if (!c) return PSG_ENOMEM;
  c->cfg = *cfg;
  c->W = (cfg->n + 63) / 64;
  c->cap = cfg->batch_capacity;
  const int nd = cfg->n_devices;
  for (int d = 0; d < nd; ++d) {
    psg_config sc = *cfg;
    sc.n_devices = 0;
    sc.device = cfg->devices[d];
    sc.batch_capacity = (cfg->batch_capacity + nd - 1) / nd;
    psg_ctx* sub = nullptr;
    const int rc = psg_create(&sub, &sc);
    if (rc) {
      g_create_err = "device " + std::to_string(cfg->devices[d]) + ": " + g_create_err;
      psg_destroy(c);
      return rc;
    }
    c->subs.push_back(sub);
  }
  *out = c;
  return PSG_OK;
}

int psg_create(psg_ctx** out, const psg_config* cfg) {
  if (!out) return PSG_EINVAL;
  *out = nullptr;
  std::string m;
  int rc = validate(cfg, m);
  if (rc) { g_create_err = m; return rc; }
  if (cfg->n_devices > 0) return create_multi(out, cfg);
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) { g_create_err = "no HIP device"; return PSG_ENODEV; }
  if (cfg->device < 0 || cfg->device >= ndev) { g_create_err = "device ordinal out of range"; return PSG_ENODEV; }
  psg_ctx* c = new (std::nothrow) psg_ctx();
  if (!c) return PSG_ENOMEM;
  c->cfg = *cfg;
  c->W = (cfg->n + 63) / 64;
  c->cap = cfg->batch_capacity;
  auto bail = [&](hipError_t err, const char* what) {
    g_create_err = std::string(what) + ": " + hipGetErrorString(err);
    psg_destroy(c);
    return err == hipErrorOutOfMemory ? PSG_ENOMEM : PSG_EIO;
  };
#define CK(call) do { hipError_t e_ = (call); if (e_ != hipSuccess) return bail(e_, #call); } while (0)
  CK(hipSetDevice(cfg->device));
  CK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  CK(hipEventCreate(&c->ev0));
  CK(hipEventCreate(&c->ev1));
  const uint64_t cells = c->cap * (uint64_t)cfg->n;
  if (cfg->alg == PSG_ALG_EPSILON) {
    CK(hipMalloc(&c->d_init_f64, sizeof(double) * cells));
    CK(hipMalloc(&c->d_dec_f64, sizeof(double) * cells));
  } else {
    CK(hipMalloc(&c->d_init, sizeof(int32_t) * cells));
  }
  CK(hipMalloc(&c->d_dec, sizeof(int32_t) * cells));
  CK(hipMalloc(&c->d_dround, sizeof(uint8_t) * cells));
  CK(hipMalloc(&c->d_inst, sizeof(psg_instance_summary) * c->cap));
  CK(hipMalloc(&c->d_counters, sizeof(unsigned long long) * NCOUNTERS_ALLOC));
  if (cfg->alg == PSG_ALG_KSET && c->W > 1)  // 520 + 4n bytes per batch row (psg_kset.hip hand-off)
    CK(hipMalloc(&c->d_hand, sizeof(uint64_t) * 65 * c->cap + sizeof(int32_t) * cells));
  const void* kp = kernel_ptr(cfg->alg, c->W);
  int per_cu = 0;
  const int threads = c->W == 1 ? 256 : 64 * c->W;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kp, threads, 0));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, cfg->device));
  if (per_cu < 1) per_cu = 1;
  c->grid_max = prop.multiProcessorCount * per_cu;
#undef CK
  *out = c;
  return PSG_OK;
}

// multi-device psg_load_inputs / _f64: each device stages its slice
static int multi_load_inputs(psg_ctx* c, uint64_t inst_begin, uint64_t count, const int32_t* host_init,
                             const double* host_f64, bool f64) {
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  const uint64_t n = (uint64_t)c->cfg.n, nd = c->subs.size();
  const int rc = par_subs(c, [&](size_t d) {
    uint64_t off, m;
    split(count, nd, d, off, m);
    return f64 ? psg_load_inputs_f64(c->subs[d], inst_begin + off, m, host_f64 ? host_f64 + off * n : nullptr)
               : psg_load_inputs(c->subs[d], inst_begin + off, m, host_init ? host_init + off * n : nullptr);
  });
  if (rc) return rc;
  c->staged = true;
  c->staged_host = f64 ? host_f64 != nullptr : host_init != nullptr;
  c->staged_begin = inst_begin;
  c->staged_count = count;
  return PSG_OK;
}

int psg_load_inputs(psg_ctx* c, uint64_t inst_begin, uint64_t count, const int32_t* host_init) {
  if (!c) return PSG_EINVAL;
  if (!c->subs.empty()) {
    if (c->cfg.alg == PSG_ALG_EPSILON && host_init)
      return fail(c, PSG_EINVAL, "EpsilonConsensus takes Double inputs: use psg_load_inputs_f64");
    return multi_load_inputs(c, inst_begin, count, host_init, nullptr, c->cfg.alg == PSG_ALG_EPSILON);
  }
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  if (c->cfg.alg == PSG_ALG_EPSILON) {
    if (host_init) return fail(c, PSG_EINVAL, "EpsilonConsensus takes Double inputs: use psg_load_inputs_f64");
    return psg_load_inputs_f64(c, inst_begin, count, nullptr);
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t cells = count * (uint64_t)c->cfg.n;
  if (host_init) {
    HIPCHK(c, hipMemcpyAsync(c->d_init, host_init, sizeof(int32_t) * cells, hipMemcpyHostToDevice, c->stream));
  } else {
    HIPCHK(c, launch_gen_init(inst_begin, count, c->cfg.n, c->cfg.alg, c->cfg.value_range, c->cfg.seed, c->d_init,
                              c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->staged = true;
  c->staged_host = host_init != nullptr;
  c->staged_begin = inst_begin;
  c->staged_count = count;
  return PSG_OK;
}

int psg_load_inputs_f64(psg_ctx* c, uint64_t inst_begin, uint64_t count, const double* host_init) {
  if (!c) return PSG_EINVAL;
  if (c->cfg.alg != PSG_ALG_EPSILON) return fail(c, PSG_EINVAL, "Double inputs are for EpsilonConsensus only");
  if (!c->subs.empty()) return multi_load_inputs(c, inst_begin, count, nullptr, host_init, true);
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (host_init) {
    const uint64_t cells = count * (uint64_t)c->cfg.n;
    HIPCHK(c, hipMemcpyAsync(c->d_init_f64, host_init, sizeof(double) * cells, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  c->init_f64_host = host_init != nullptr;
  c->staged = true;
  c->staged_host = host_init != nullptr;
  c->staged_begin = inst_begin;
  c->staged_count = count;
  return PSG_OK;
}

// multi-device psg_run_batch / psg_run_batch_spec (prog != nullptr)
static int multi_run(psg_ctx* c, uint64_t inst_begin, uint64_t count, const psg_spec_program* prog, psg_summary* out,
                     psg_instance_summary* per_inst) {
  if (out) std::memset(out, 0, sizeof(*out));
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  if (count == 0) {  // the library's "last batch" is the single source of truth (JNI checks use it)
    c->last_count = 0;
    for (psg_ctx* s : c->subs) s->last_count = 0;
    return PSG_OK;
  }
  if (c->ho_loaded && (inst_begin != c->ho_begin || count != c->ho_count))
    return fail(c, PSG_ERANGE, "a multi-device run under an explicit schedule covers exactly the loaded range");
  if (!(c->staged && c->staged_begin == inst_begin && c->staged_count == count)) {
    const int rc = psg_load_inputs(c, inst_begin, count, nullptr);  // seeded, like a single device
    if (rc) return rc;
  }
  const size_t nd = c->subs.size();
  std::vector<psg_summary> parts(nd);
  const int rc = par_subs(c, [&](size_t d) {
    uint64_t off, m;
    split(count, nd, d, off, m);
    psg_instance_summary* pi = per_inst ? per_inst + off : nullptr;
    return prog ? psg_run_batch_spec(c->subs[d], inst_begin + off, m, prog, &parts[d], pi)
                : psg_run_batch(c->subs[d], inst_begin + off, m, &parts[d], pi);
  });
  if (rc) return rc;
  if (out)
    for (size_t d = 0; d < nd; ++d) summary_add(*out, parts[d]);
  c->last_count = count;
  return PSG_OK;
}

int psg_run_batch(psg_ctx* c, uint64_t inst_begin, uint64_t count, psg_summary* out, psg_instance_summary* per_inst) {
  if (!c) return PSG_EINVAL;
  if (!c->subs.empty()) return multi_run(c, inst_begin, count, nullptr, out, per_inst);
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  if (count == 0) {
    if (out) std::memset(out, 0, sizeof(*out));
    c->last_count = 0;
    return PSG_OK;
  }
  if (int rc = check_sched_range(c, inst_begin, count)) return rc;
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (!(c->staged && c->staged_begin == inst_begin && c->staged_count == count)) {
    int rc = psg_load_inputs(c, inst_begin, count, nullptr);
    if (rc) return rc;
  }
  KArgs a = make_args(c);
  a.inst_begin = inst_begin;
  a.count = count;
  a.init = c->d_init;
  if (c->cfg.alg == PSG_ALG_EPSILON) {
    a.init = nullptr;
    a.init_f64 = c->init_f64_host ? c->d_init_f64 : nullptr;  // else seeded inside the kernel
    a.out_dec_f64 = c->d_dec_f64;
  }
  a.out_decision = c->d_dec;
  a.out_dround = c->d_dround;
  a.out_inst = c->d_inst;
  int rc = run_kernel(c, a, count, out, true);
  if (rc) return rc;
  c->last_count = count;
  if (per_inst) {
    HIPCHK(c, hipMemcpy(per_inst, c->d_inst, sizeof(psg_instance_summary) * count, hipMemcpyDeviceToHost));
  }
  return PSG_OK;
}

static int validate_prog(const psg_spec_program* p, std::string& m) {
  if (!p || !p->code || !p->slot_entry || !p->slot_flags) { m = "null spec program"; return PSG_EINVAL; }
  if (p->n_slots < 1 || p->n_slots > PSG_MAX_CHECKS) { m = "spec program needs 1..12 slots"; return PSG_EINVAL; }
  if (p->n_words < 1 || p->n_words > (1 << 20)) { m = "bad spec program length"; return PSG_EINVAL; }
  if (p->n_vars < 0 || p->n_vars > 16) { m = "spec program uses more than 16 bound variables"; return PSG_EINVAL; }
  for (int s = 0; s < p->n_slots; ++s)
    if (p->slot_entry[s] < 0 || p->slot_entry[s] >= p->n_words) { m = "slot entry out of range"; return PSG_EINVAL; }
  if (p->term_entry >= p->n_words) { m = "termination entry out of range"; return PSG_EINVAL; }
  // structural check: opcodes known, quantifier ends in range, variables in range
  for (int pc = 0; pc < p->n_words;) {
    const int32_t w = p->code[pc];
    const int op = w & 0xff, a = (w >> 8) & 0xff;
    if (op > PSG_OP_COORD) { m = "unknown opcode at " + std::to_string(pc); return PSG_EINVAL; }
    if ((op == PSG_OP_VAR || op == PSG_OP_BIND) && a >= 16) { m = "variable out of range"; return PSG_EINVAL; }
    if (op == PSG_OP_FIELD && (a >= PSG_NFIELDS || (w >> 16) < 0 || (w >> 16) > PSG_TAG_INIT)) {
      m = "bad field / tag at " + std::to_string(pc);
      return PSG_EINVAL;
    }
    ++pc;
    if (op == PSG_OP_IMM32) ++pc;
    if (op == PSG_OP_QBEGIN) {
      if (a > PSG_Q_EXISTS_VI || (w >> 16) < 0 || (w >> 16) >= 16 || pc >= p->n_words) {
        m = "bad quantifier at " + std::to_string(pc - 1);
        return PSG_EINVAL;
      }
      const int32_t end = p->code[pc];
      if (end <= pc || end >= p->n_words || (p->code[end] & 0xff) != PSG_OP_QEND) {
        m = "quantifier end mismatch at " + std::to_string(pc - 1);
        return PSG_EINVAL;
      }
      ++pc;
      if (a == PSG_Q_EXISTS_VI) {
        if (pc >= p->n_words) { m = "truncated V.exists"; return PSG_EINVAL; }
        pc += 1 + ((p->code[pc] >> 16) & 0xffff);
      }
    }
  }
  return PSG_OK;
}

// Fields a (validated) program reads: FIELD operands and V.exists field sets.
static uint32_t prog_fields(const psg_spec_program* p) {
  uint32_t m = 0;
  for (int pc = 0; pc < p->n_words;) {
    const int32_t w = p->code[pc];
    const int op = w & 0xff, a = (w >> 8) & 0xff;
    if (op == PSG_OP_FIELD) m |= 1u << a;
    ++pc;
    if (op == PSG_OP_IMM32) ++pc;
    if (op == PSG_OP_QBEGIN) {
      ++pc;
      if (a == PSG_Q_EXISTS_VI) {
        const int nf = (p->code[pc] >> 16) & 0xffff;
        for (int k = 0; k < nf; ++k) m |= 1u << (p->code[pc + 1 + k] & 0xff);
        pc += 1 + nf;
      }
    }
  }
  return m & ((1u << PSG_NFIELDS) - 1u);
}

int psg_last_batch_count(const psg_ctx* c, uint64_t* count) {
  if (!c || !count) return PSG_EINVAL;
  *count = c->last_count;
  return PSG_OK;
}

int psg_copy_decisions(psg_ctx* c, int32_t* decision, int32_t* decision_round) {
  if (!c) return PSG_EINVAL;
  if (!c->subs.empty()) {  // the last batch's slices, in device order
    const uint64_t n = (uint64_t)c->cfg.n, nd = c->subs.size();
    for (size_t d = 0; d < nd; ++d) {
      uint64_t off, m;
      split(c->last_count, nd, d, off, m);
      if (!m) continue;  // an empty slice: the device ran nothing (its own last_count is 0)
      const int rc = psg_copy_decisions(c->subs[d], decision ? decision + off * n : nullptr,
                                        decision_round ? decision_round + off * n : nullptr);
      if (rc) return fail(c, rc, "device " + std::to_string(c->cfg.devices[d]) + ": " + c->subs[d]->err);
    }
    return PSG_OK;
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t cells = c->last_count * (uint64_t)c->cfg.n;
  if (decision) HIPCHK(c, hipMemcpy(decision, c->d_dec, sizeof(int32_t) * cells, hipMemcpyDeviceToHost));
  if (decision_round) {
    uint8_t* tmp = new (std::nothrow) uint8_t[cells ? cells : 1];
    if (!tmp) return fail(c, PSG_ENOMEM, "host allocation failed");
    hipError_t e = hipMemcpy(tmp, c->d_dround, cells, hipMemcpyDeviceToHost);
    if (e != hipSuccess) { delete[] tmp; return hip_fail(c, e, "hipMemcpy(dround)"); }
    for (uint64_t k = 0; k < cells; ++k) decision_round[k] = tmp[k] == 0xFF ? -1 : (int32_t)tmp[k];
    delete[] tmp;
  }
  return PSG_OK;
}

int psg_run_batch_spec(psg_ctx* c, uint64_t inst_begin, uint64_t count, const psg_spec_program* prog,
                       psg_summary* out, psg_instance_summary* per_inst) {
  if (!c) return PSG_EINVAL;
  if (c->cfg.alg == PSG_ALG_EPSILON) return fail(c, PSG_EINVAL, "Spec programs need integer state (not EpsilonConsensus)");
  std::string m;
  if (validate_prog(prog, m)) return fail(c, PSG_EINVAL, m);
  if (prog->alg != 0 && prog->alg != c->cfg.alg)
    return fail(c, PSG_EINVAL, "spec program was compiled for algorithm " + std::to_string(prog->alg) +
                                   ", the context runs " + std::to_string(c->cfg.alg));
  if (!c->subs.empty()) return multi_run(c, inst_begin, count, prog, out, per_inst);
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  if (int rc = check_sched_range(c, inst_begin, count)) return rc;
  if (out) std::memset(out, 0, sizeof(*out));
  if (count == 0) {
    c->last_count = 0;
    return PSG_OK;
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const int n = c->cfg.n, R = c->cfg.rounds;
  // program: code | slot_entry | slot_flags
  const size_t words = (size_t)prog->n_words + 2 * (size_t)prog->n_slots;
  if (words > c->prog_cap) {
    if (c->d_prog) (void)hipFree(c->d_prog);
    c->d_prog = nullptr;
    c->prog_cap = 0;
    HIPCHK(c, hipMalloc(&c->d_prog, sizeof(int32_t) * words));
    c->prog_cap = words;
  }
  HIPCHK(c, hipMemcpy(c->d_prog, prog->code, sizeof(int32_t) * prog->n_words, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_prog + prog->n_words, prog->slot_entry, sizeof(int32_t) * prog->n_slots,
                      hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(c->d_prog + prog->n_words + prog->n_slots, prog->slot_flags, sizeof(int32_t) * prog->n_slots,
                      hipMemcpyHostToDevice));
  // native lowering of the same Spec (round_amd/formula.py compile_native), if given
  const bool native = prog->module_path != nullptr;
  if (native && c->module_path != prog->module_path) {
    if (c->module) (void)hipModuleUnload(c->module);
    c->module = nullptr;
    c->native_fn = nullptr;
    c->fused_fn = c->fused_x_fn = nullptr;
    c->module_path.clear();
    HIPCHK(c, hipModuleLoad(&c->module, prog->module_path));
    const std::string name = "psg_spec_native_w" + std::to_string(c->W);
    HIPCHK(c, hipModuleGetFunction(&c->native_fn, c->module, name.c_str()));
    // the algorithm the module was generated for (round_amd/formula.py writes psg_spec_alg)
    c->module_alg = 0;
    hipDeviceptr_t gp = nullptr;
    size_t gsz = 0;
    if (hipModuleGetGlobal(&gp, &gsz, c->module, "psg_spec_alg") == hipSuccess && gsz == sizeof(int32_t))
      HIPCHK(c, hipMemcpyDtoH(&c->module_alg, gp, sizeof(int32_t)));
    (void)hipGetLastError();
    // fused modules (compile_native(fused=True)) also hold the round kernel with the Spec as its hook
    const std::string aw = "a" + std::to_string(c->cfg.alg) + "_w" + std::to_string(c->W);
    const std::string fw = "psg_fused_" + aw, fx = "psg_fused_x_" + aw;
    if (hipModuleGetFunction(&c->fused_fn, c->module, fw.c_str()) != hipSuccess) c->fused_fn = nullptr;
    if (hipModuleGetFunction(&c->fused_x_fn, c->module, fx.c_str()) != hipSuccess) c->fused_x_fn = nullptr;
    (void)hipGetLastError();
    c->module_path = prog->module_path;
  }
  if (native && c->module_alg != 0 && c->module_alg != c->cfg.alg)
    return fail(c, PSG_EINVAL, "spec module " + c->module_path + " was generated for algorithm " +
                                   std::to_string(c->module_alg) + ", the context runs " + std::to_string(c->cfg.alg));
  if (native && (c->ho_loaded ? c->fused_x_fn : c->fused_fn)) {
    // one launch: rounds + Spec from registers (no trace, no chunks)
    hipFunction_t fn = c->ho_loaded ? c->fused_x_fn : c->fused_fn;
    if (!(c->staged && c->staged_begin == inst_begin && c->staged_count == count)) {
      int rc = psg_load_inputs(c, inst_begin, count, nullptr);
      if (rc) return rc;
    }
    KArgs a = make_args(c);
    a.inst_begin = inst_begin;
    a.count = count;
    a.init = c->d_init;
    a.out_decision = c->d_dec;
    a.out_dround = c->d_dround;
    a.out_inst = c->d_inst;
    const int threads = c->W == 1 ? 256 : 64 * c->W;
    int per_cu = 0, cus = 0;
    HIPCHK(c, hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, threads, 0));
    HIPCHK(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->cfg.device));
    const int G = groups_per_block(c->W);
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((count + G - 1) / G,
                                                                           (uint64_t)cus * std::max(per_cu, 1)));
    HIPCHK(c, hipMemsetAsync(c->d_counters, 0, sizeof(unsigned long long) * NCOUNTERS_ALLOC, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    void* params[] = {&a};
    HIPCHK(c, hipModuleLaunchKernel(fn, grid, 1, 1, (unsigned)threads, 1, 1, 0, c->stream, params, nullptr));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    unsigned long long host[NCOUNTERS_ALLOC];
    HIPCHK(c, hipMemcpyAsync(host, c->d_counters, sizeof(host), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    // a fused module compiled with -DPSG_PHASE_TIMERS=1 (formula.compile_native(defines=...)) run
    // through a profiling build of the library
    if (PSG_PHASE_TIMERS && std::getenv("PSG_PHASE_TIMERS")) print_timers(host);
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (out) {
      out->instances = (int64_t)count;
      out->process_rounds = (int64_t)count * c->cfg.n * c->cfg.rounds;
      out->active_process_rounds = (int64_t)host[C_ACTIVE];
      out->live_instance_rounds = (int64_t)host[C_LIVE];
      for (int i = 0; i < PSG_MAX_CHECKS; ++i) out->fail_count[i] = (int64_t)host[C_FAIL + i];
      out->decided_processes = (int64_t)host[C_DECIDED];
      out->digest = (int64_t)host[C_DIGEST];
      for (int i = 0; i < R + 2; ++i) out->term_hist[i] = (int64_t)host[C_HIST + i];
      out->kernel_ns = (int64_t)((double)ms * 1e6);
    }
    c->last_count = count;
    if (per_inst)
      HIPCHK(c, hipMemcpy(per_inst, c->d_inst, sizeof(psg_instance_summary) * count, hipMemcpyDeviceToHost));
    return PSG_OK;
  }
  // trace chunk: <= PSG_SPEC_TRACE_MB (default 2048) MiB of [R+1][fields][n] int32 rows
  uint64_t budget = 2048ull << 20;
  if (const char* e = std::getenv("PSG_SPEC_TRACE_MB")) {
    const long long mb = std::atoll(e);
    if (mb > 0) budget = (uint64_t)mb << 20;
  }
  const uint64_t per_inst_bytes = (uint64_t)(R + 1) * PSG_NFIELDS * (uint64_t)n * sizeof(int32_t);
  const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(count, budget / per_inst_bytes));
  if (chunk > c->trace_cap) {
    if (c->d_trace) (void)hipFree(c->d_trace);
    c->d_trace = nullptr;
    c->trace_cap = 0;
    HIPCHK(c, hipMalloc(&c->d_trace, per_inst_bytes * chunk));
    c->trace_cap = chunk;
  }
  if (!c->d_vm_counters) HIPCHK(c, hipMalloc(&c->d_vm_counters, sizeof(unsigned long long) * NCOUNTERS));
  if (!c->d_vm_err) HIPCHK(c, hipMalloc(&c->d_vm_err, sizeof(int32_t)));
  HIPCHK(c, hipMemsetAsync(c->d_vm_err, 0, sizeof(int32_t), c->stream));
  const bool staged = c->staged && c->staged_begin == inst_begin && c->staged_count == count;
  const uint32_t fields = prog_fields(prog);
  psg_summary acc;
  std::memset(&acc, 0, sizeof(acc));
  int vm_grid = 0;
  HIPCHK(c, hipDeviceGetAttribute(&vm_grid, hipDeviceAttributeMultiprocessorCount, c->cfg.device));
  vm_grid *= 8;
  for (uint64_t off = 0; off < count; off += chunk) {
    const uint64_t m_cnt = std::min<uint64_t>(chunk, count - off);
    KArgs a = make_args(c);
    a.inst_begin = inst_begin + off;
    a.count = m_cnt;
    a.init = staged ? c->d_init + off * (uint64_t)n : nullptr;  // else seeded by the kernel
    a.out_decision = c->d_dec + off * (uint64_t)n;
    a.out_dround = c->d_dround + off * (uint64_t)n;
    a.out_inst = c->d_inst + off;
    a.trace = c->d_trace;
    a.trace_fields = fields;
    psg_summary part;
    int rc = run_kernel(c, a, m_cnt, &part, true);
    if (rc) return rc;
    VmArgs v;
    v.code = c->d_prog;
    v.slot_entry = c->d_prog + prog->n_words;
    v.slot_flags = c->d_prog + prog->n_words + prog->n_slots;
    v.n_slots = prog->n_slots;
    v.term_entry = prog->term_entry;
    v.n_words = prog->n_words;
    v.trace = c->d_trace;
    v.count = m_cnt;
    v.n = n;
    v.R = R;
    v.out_inst = c->d_inst + off;
    v.counters = c->d_vm_counters;
    v.err = c->d_vm_err;
    HIPCHK(c, hipMemsetAsync(c->d_vm_counters, 0, sizeof(unsigned long long) * NCOUNTERS, c->stream));
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    if (native) {
      const int G = groups_per_block(c->W);
      const unsigned grid = (unsigned)std::min<uint64_t>((m_cnt + G - 1) / G, (uint64_t)vm_grid);
      const unsigned threads = c->W == 1 ? 256u : 64u * (unsigned)c->W;
      void* params[] = {&v};
      HIPCHK(c, hipModuleLaunchKernel(c->native_fn, grid, 1, 1, threads, 1, 1, 0, c->stream, params, nullptr));
    } else {
      HIPCHK(c, launch_spec_vm(v, (int)std::min<uint64_t>(m_cnt, (uint64_t)vm_grid), c->stream));
    }
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    unsigned long long host[NCOUNTERS];
    HIPCHK(c, hipMemcpyAsync(host, c->d_vm_counters, sizeof(host), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    acc.instances += part.instances;
    acc.process_rounds += part.process_rounds;
    acc.active_process_rounds += part.active_process_rounds;
    acc.live_instance_rounds += part.live_instance_rounds;
    acc.decided_processes += part.decided_processes;
    acc.digest = (int64_t)((uint64_t)acc.digest + (uint64_t)part.digest);
    acc.kernel_ns += part.kernel_ns + (int64_t)((double)ms * 1e6);
    for (int i = 0; i < PSG_MAX_CHECKS; ++i) acc.fail_count[i] += (int64_t)host[C_FAIL + i];
    for (int i = 0; i < R + 2; ++i) acc.term_hist[i] += (int64_t)host[C_HIST + i];
  }
  int32_t verr = 0;
  HIPCHK(c, hipMemcpy(&verr, c->d_vm_err, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (verr) {
    return fail(c, PSG_ERANGE,
                std::string("spec program exceeded interpreter limits (flags ") + std::to_string(verr) +
                    "; 1 stack > 24, 2 nesting > 12, 4 V.exists candidates > 1024 or nesting > 2, 8 bad opcode)");
  }
  c->last_count = count;
  if (per_inst)
    HIPCHK(c, hipMemcpy(per_inst, c->d_inst, sizeof(psg_instance_summary) * count, hipMemcpyDeviceToHost));
  if (out) *out = acc;
  return PSG_OK;
}

int psg_copy_decisions_f64(psg_ctx* c, double* decision, int32_t* decision_round) {
  if (!c) return PSG_EINVAL;
  if (c->cfg.alg != PSG_ALG_EPSILON) return fail(c, PSG_EINVAL, "Double decisions are for EpsilonConsensus only");
  if (!c->subs.empty()) {
    const uint64_t n = (uint64_t)c->cfg.n, nd = c->subs.size();
    for (size_t d = 0; d < nd; ++d) {
      uint64_t off, m;
      split(c->last_count, nd, d, off, m);
      if (!m) continue;
      const int rc = psg_copy_decisions_f64(c->subs[d], decision ? decision + off * n : nullptr,
                                            decision_round ? decision_round + off * n : nullptr);
      if (rc) return fail(c, rc, "device " + std::to_string(c->cfg.devices[d]) + ": " + c->subs[d]->err);
    }
    return PSG_OK;
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t cells = c->last_count * (uint64_t)c->cfg.n;
  if (decision) HIPCHK(c, hipMemcpy(decision, c->d_dec_f64, sizeof(double) * cells, hipMemcpyDeviceToHost));
  return decision_round ? psg_copy_decisions(c, nullptr, decision_round) : PSG_OK;
}

static int fetch_impl(psg_ctx* c, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                      psg_process_record* procs, double* fdec, double* fx, bool force_seeded = false);

// multi-device fetch: each id goes to the device holding its schedule slice (explicit
// schedule) or its staged host-input slice; otherwise ids are dealt out in contiguous
// chunks and re-executed from seeded inputs (what staged seeded rows hold anyway).
static int multi_fetch(psg_ctx* c, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                       psg_process_record* procs, double* fdec, double* fx) {
  if (k > c->cap) return fail(c, PSG_ERANGE, "fetch count exceeds batch_capacity");
  const size_t nd = c->subs.size();
  const uint64_t n = (uint64_t)c->cfg.n;
  bool all_staged = c->staged && c->staged_host;
  for (size_t j = 0; j < k && all_staged; ++j)
    all_staged = ids[j] >= c->staged_begin && ids[j] - c->staged_begin < c->staged_count;
  auto owner = [&](uint64_t id, uint64_t begin, uint64_t count) {  // device whose slice holds id
    size_t d = (size_t)((id - begin) * nd / count);
    uint64_t off, m;
    for (;; ++d) {
      split(count, nd, d, off, m);
      if (id - begin < off + m || d + 1 == nd) return d;
    }
  };
  std::vector<std::vector<size_t>> pos(nd);
  for (size_t j = 0; j < k; ++j) {
    size_t d;
    if (c->ho_loaded) {
      if (ids[j] < c->ho_begin || ids[j] - c->ho_begin >= c->ho_count)
        return fail(c, PSG_ERANGE, "instances outside the loaded explicit schedule");
      if (all_staged && (c->staged_begin != c->ho_begin || c->staged_count != c->ho_count))
        return fail(c, PSG_EINVAL, "multi-device fetch: staged host inputs and the explicit schedule cover different ranges");
      d = owner(ids[j], c->ho_begin, c->ho_count);
    } else if (all_staged) {
      d = owner(ids[j], c->staged_begin, c->staged_count);
    } else {
      d = j * nd / k;
    }
    pos[d].push_back(j);
  }
  return par_subs(c, [&](size_t d) {
    psg_ctx* s = c->subs[d];
    const std::vector<size_t>& P = pos[d];
    const size_t chunk = (size_t)std::max<uint64_t>(1, s->cap);
    std::vector<uint64_t> sid;
    std::vector<psg_instance_summary> ss;
    std::vector<psg_process_record> sp;
    std::vector<double> sd, sx;
    for (size_t a = 0; a < P.size(); a += chunk) {
      const size_t m = std::min(chunk, P.size() - a);
      sid.resize(m);
      for (size_t t = 0; t < m; ++t) sid[t] = ids[P[a + t]];
      ss.resize(m);
      if (procs) sp.resize(m * n);
      if (fdec) sd.resize(m * n);
      if (fx) sx.resize(m * n);
      const int rc = fetch_impl(s, sid.data(), m, ss.data(), procs ? sp.data() : nullptr, fdec ? sd.data() : nullptr,
                                fx ? sx.data() : nullptr, !all_staged);
      if (rc) return rc;
      for (size_t t = 0; t < m; ++t) {
        const size_t j = P[a + t];
        if (sums) sums[j] = ss[t];
        if (procs) std::memcpy(procs + j * n, sp.data() + t * n, sizeof(psg_process_record) * n);
        if (fdec) std::memcpy(fdec + j * n, sd.data() + t * n, sizeof(double) * n);
        if (fx) std::memcpy(fx + j * n, sx.data() + t * n, sizeof(double) * n);
      }
    }
    return PSG_OK;
  });
}

int psg_fetch_instances(psg_ctx* c, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                        psg_process_record* procs) {
  if (c && !c->subs.empty()) {
    if (!ids && k) return PSG_EINVAL;
    return multi_fetch(c, ids, k, sums, procs, nullptr, nullptr);
  }
  return fetch_impl(c, ids, k, sums, procs, nullptr, nullptr);
}

int psg_fetch_instances_f64(psg_ctx* c, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                            psg_process_record* procs, double* decision, double* final_x) {
  if (c && c->cfg.alg != PSG_ALG_EPSILON) return fail(c, PSG_EINVAL, "Double records are for EpsilonConsensus only");
  if (c && !c->subs.empty()) {
    if (!ids && k) return PSG_EINVAL;
    return multi_fetch(c, ids, k, sums, procs, decision, final_x);
  }
  return fetch_impl(c, ids, k, sums, procs, decision, final_x);
}

static int fetch_impl(psg_ctx* c, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                      psg_process_record* procs, double* fdec, double* fx, bool force_seeded) {
  if (!c || (!ids && k)) return PSG_EINVAL;
  if (k == 0) return PSG_OK;
  if (k > c->cap) return fail(c, PSG_ERANGE, "fetch count exceeds batch_capacity");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (k > c->fetch_cap) {
    if (c->d_ids) (void)hipFree(c->d_ids);
    if (c->d_rec) (void)hipFree(c->d_rec);
    c->d_ids = nullptr;
    c->d_rec = nullptr;
    c->fetch_cap = 0;
    HIPCHK(c, hipMalloc(&c->d_ids, sizeof(uint64_t) * k));
    HIPCHK(c, hipMalloc(&c->d_rec, sizeof(psg_process_record) * k * (uint64_t)c->cfg.n));
    if (c->cfg.alg == PSG_ALG_EPSILON) {
      if (c->d_rec_f64) (void)hipFree(c->d_rec_f64);
      c->d_rec_f64 = nullptr;
      HIPCHK(c, hipMalloc(&c->d_rec_f64, sizeof(double) * 2 * k * (uint64_t)c->cfg.n));
    }
    c->fetch_cap = k;
  }
  bool in_staged = c->staged && !force_seeded;
  for (size_t j = 0; j < k; ++j) {
    if (int rc = check_sched_range(c, ids[j], 1)) return rc;
    if (ids[j] < c->staged_begin || ids[j] - c->staged_begin >= c->staged_count) in_staged = false;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_ids, ids, sizeof(uint64_t) * k, hipMemcpyHostToDevice, c->stream));
  KArgs a = make_args(c);
  a.inst_begin = 0;
  a.count = k;
  a.ids = c->d_ids;
  // inputs of each listed id: the staged rows when all ids are staged, else seeded
  a.init = nullptr;
  if (in_staged) {
    a.init_base = c->staged_begin;
    if (c->cfg.alg == PSG_ALG_EPSILON) a.init_f64 = c->init_f64_host ? c->d_init_f64 : nullptr;
    else a.init = c->d_init;
  }
  a.out_inst = c->d_inst;
  a.out_rec = c->d_rec;
  a.out_rec_f64 = c->d_rec_f64;
  int rc = run_kernel(c, a, k, nullptr, false);
  if (rc) return rc;
  if (fdec || fx) {
    const uint64_t cells = k * (uint64_t)c->cfg.n;
    double* tmp = new (std::nothrow) double[2 * cells];
    if (!tmp) return fail(c, PSG_ENOMEM, "host allocation failed");
    hipError_t e = hipMemcpy(tmp, c->d_rec_f64, sizeof(double) * 2 * cells, hipMemcpyDeviceToHost);
    if (e != hipSuccess) { delete[] tmp; return hip_fail(c, e, "hipMemcpy(rec_f64)"); }
    for (uint64_t j = 0; j < cells; ++j) {
      if (fdec) fdec[j] = tmp[2 * j];
      if (fx) fx[j] = tmp[2 * j + 1];
    }
    delete[] tmp;
  }
  if (sums) HIPCHK(c, hipMemcpy(sums, c->d_inst, sizeof(psg_instance_summary) * k, hipMemcpyDeviceToHost));
  if (procs)
    HIPCHK(c, hipMemcpy(procs, c->d_rec, sizeof(psg_process_record) * k * (uint64_t)c->cfg.n, hipMemcpyDeviceToHost));
  return PSG_OK;
}

int psg_load_schedule(psg_ctx* c, uint64_t inst_begin, uint64_t count, const uint64_t* ho,
                      const int32_t* crash_round) {
  if (!c) return PSG_EINVAL;
  if (!ho && count) return fail(c, PSG_EINVAL, "null schedule");
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  if (!c->subs.empty()) {
    const uint64_t per = (uint64_t)c->cfg.rounds * (uint64_t)c->cfg.n * (uint64_t)c->W, nd = c->subs.size();
    const int rc = par_subs(c, [&](size_t d) {
      uint64_t off, m;
      split(count, nd, d, off, m);
      return psg_load_schedule(c->subs[d], inst_begin + off, m, ho ? ho + off * per : nullptr,
                               crash_round ? crash_round + off * (uint64_t)c->cfg.n : nullptr);
    });
    if (rc) return rc;
    c->ho_loaded = true;
    c->ho_has_crash = crash_round != nullptr;
    c->ho_begin = inst_begin;
    c->ho_count = count;
    return PSG_OK;
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t n = (uint64_t)c->cfg.n, R = (uint64_t)c->cfg.rounds, W = (uint64_t)c->W;
  if (count > c->ho_cap) {
    if (c->d_ho) (void)hipFree(c->d_ho);
    if (c->d_crash) (void)hipFree(c->d_crash);
    c->d_ho = nullptr;
    c->d_crash = nullptr;
    c->ho_cap = 0;
    c->ho_loaded = false;
    HIPCHK(c, hipMalloc(&c->d_ho, sizeof(uint64_t) * count * R * n * W));
    HIPCHK(c, hipMalloc(&c->d_crash, sizeof(int32_t) * count * n));
    c->ho_cap = count;
  }
  if (count) {
    HIPCHK(c, hipMemcpyAsync(c->d_ho, ho, sizeof(uint64_t) * count * R * n * W, hipMemcpyHostToDevice, c->stream));
    if (crash_round)
      HIPCHK(c, hipMemcpyAsync(c->d_crash, crash_round, sizeof(int32_t) * count * n, hipMemcpyHostToDevice,
                               c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  c->ho_loaded = true;
  c->ho_has_crash = crash_round != nullptr;
  c->ho_begin = inst_begin;
  c->ho_count = count;
  return PSG_OK;
}

int psg_clear_schedule(psg_ctx* c) {
  if (!c) return PSG_EINVAL;
  for (psg_ctx* s : c->subs) (void)psg_clear_schedule(s);
  c->ho_loaded = false;
  c->ho_has_crash = false;
  c->ho_begin = c->ho_count = 0;
  return PSG_OK;
}

int psg_materialize_schedule(psg_ctx* c, uint64_t inst_begin, uint64_t count, uint64_t* ho, int32_t* crash_round) {
  if (!c) return PSG_EINVAL;
  if (!ho && count) return fail(c, PSG_EINVAL, "null output");
  if (count == 0) return PSG_OK;
  if (!c->subs.empty()) {
    const uint64_t per = (uint64_t)c->cfg.rounds * (uint64_t)c->cfg.n * (uint64_t)c->W, nd = c->subs.size();
    return par_subs(c, [&](size_t d) {
      uint64_t off, m;
      split(count, nd, d, off, m);
      return m ? psg_materialize_schedule(c->subs[d], inst_begin + off, m, ho + off * per,
                                          crash_round ? crash_round + off * (uint64_t)c->cfg.n : nullptr)
               : PSG_OK;
    });
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t n = (uint64_t)c->cfg.n, R = (uint64_t)c->cfg.rounds, W = (uint64_t)c->W;
  const uint64_t per = R * n * W * sizeof(uint64_t);
  const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(count, (256ull << 20) / per));
  uint64_t* d_out = nullptr;
  int32_t* d_cr = nullptr;
  hipError_t e = hipMalloc(&d_out, per * chunk);
  if (e == hipSuccess) e = hipMalloc(&d_cr, sizeof(int32_t) * n * chunk);
  int rc = PSG_OK;
  KArgs a = make_args(c);
  a.ho_in = nullptr;  // always the seeded generator
  a.crash_in = nullptr;
  const int G = groups_per_block(c->W);
  for (uint64_t off = 0; e == hipSuccess && off < count; off += chunk) {
    const uint64_t m = std::min<uint64_t>(chunk, count - off);
    a.inst_begin = inst_begin + off;
    a.count = m;
    const int grid = (int)std::min<uint64_t>((m + G - 1) / G, (uint64_t)c->grid_max);
    e = launch_schedule(a, c->W, grid, d_out, d_cr, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(ho + off * R * n * W, d_out, per * m, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && crash_round)
      e = hipMemcpyAsync(crash_round + off * n, d_cr, sizeof(int32_t) * n * m, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  }
  if (e != hipSuccess) rc = hip_fail(c, e, "psg_materialize_schedule");
  if (d_out) (void)hipFree(d_out);
  if (d_cr) (void)hipFree(d_cr);
  return rc;
}

// ---------------------------------------------------------------- search populations
static int pop_buffers(psg_ctx* c, uint64_t count) {
  const uint64_t n = (uint64_t)c->cfg.n, R = (uint64_t)c->cfg.rounds, W = (uint64_t)c->W;
  if (count > c->ho_cap) {  // the loaded-schedule buffers (psg_load_schedule's)
    if (c->d_ho) (void)hipFree(c->d_ho);
    if (c->d_crash) (void)hipFree(c->d_crash);
    c->d_ho = nullptr;
    c->d_crash = nullptr;
    c->ho_cap = 0;
    c->ho_loaded = false;
    HIPCHK(c, hipMalloc(&c->d_ho, sizeof(uint64_t) * count * R * n * W));
    HIPCHK(c, hipMalloc(&c->d_crash, sizeof(int32_t) * count * n));
    c->ho_cap = count;
  }
  if (count > c->pop_cap) {
    if (c->d_ho2) (void)hipFree(c->d_ho2);
    if (c->d_init2) (void)hipFree(c->d_init2);
    if (c->d_parent) (void)hipFree(c->d_parent);
    if (c->d_op) (void)hipFree(c->d_op);
    c->d_ho2 = nullptr;
    c->d_init2 = nullptr;
    c->d_parent = nullptr;
    c->d_op = nullptr;
    c->pop_cap = 0;
    const uint64_t cap = std::max(count, c->ho_cap);
    HIPCHK(c, hipMalloc(&c->d_ho2, sizeof(uint64_t) * cap * R * n * W));
    HIPCHK(c, hipMalloc(&c->d_init2, sizeof(int32_t) * c->cap * n));
    HIPCHK(c, hipMalloc(&c->d_parent, sizeof(uint32_t) * cap));
    HIPCHK(c, hipMalloc(&c->d_op, cap));
    c->pop_cap = cap;
  }
  return PSG_OK;
}

static int pop_check(psg_ctx* c, const psg_population_params* p) {
  if (!p) return fail(c, PSG_EINVAL, "null population parameters");
  if (c->cfg.alg == PSG_ALG_EPSILON) return fail(c, PSG_EINVAL, "populations hold int32 inputs (not EpsilonConsensus)");
  if (c->cfg.alg != PSG_ALG_BENOR && p->value_range < 1) return fail(c, PSG_EINVAL, "value_range must be >= 1");
  if (p->min_size > c->cfg.n) return fail(c, PSG_EINVAL, "min_size > n");
  return PSG_OK;
}

static PopArgs pop_args(const psg_ctx* c, const psg_population_params* p, uint64_t count) {
  PopArgs a;
  std::memset(&a, 0, sizeof(a));
  a.count = count;
  a.n = c->cfg.n;
  a.R = c->cfg.rounds;
  a.W = c->W;
  a.seed = p->seed;
  a.gen = p->generation;
  a.flips = p->flips;
  a.min_size = p->min_size;
  a.self_bit = p->self_bit;
  for (int j = 0; j < 4; ++j) a.keep[j] = p->keep_p256[j];
  a.V = p->value_range;
  a.redraw = p->redraw_p256;
  a.benor = c->cfg.alg == PSG_ALG_BENOR;
  return a;
}

int psg_population_fresh(psg_ctx* c, uint64_t inst_begin, uint64_t count, const psg_population_params* p) {
  if (!c) return PSG_EINVAL;
  if (!c->subs.empty()) return fail(c, PSG_EINVAL, "device-resident populations need a single-device context");
  if (int rc = pop_check(c, p)) return rc;
  if (count > c->cap) return fail(c, PSG_ERANGE, "inst_count exceeds batch_capacity");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  if (int rc = pop_buffers(c, std::max<uint64_t>(count, 1))) return rc;
  PopArgs a = pop_args(c, p, count);
  a.ho = c->d_ho;
  a.init = c->d_init;
  HIPCHK(c, launch_population(a, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->ho_loaded = true;
  c->ho_has_crash = false;
  c->ho_begin = inst_begin;
  c->ho_count = count;
  c->staged = true;
  c->staged_begin = inst_begin;
  c->staged_count = count;
  return PSG_OK;
}

int psg_population_next(psg_ctx* c, const uint32_t* parent, const uint8_t* op, const psg_population_params* p) {
  if (!c) return PSG_EINVAL;
  if (!c->subs.empty()) return fail(c, PSG_EINVAL, "device-resident populations need a single-device context");
  if (int rc = pop_check(c, p)) return rc;
  if (!(c->ho_loaded && c->staged && c->staged_begin == c->ho_begin && c->staged_count == c->ho_count) ||
      c->pop_cap < c->ho_count)
    return fail(c, PSG_EINVAL, "no population loaded (psg_population_fresh first)");
  const uint64_t count = c->ho_count;
  if (count && (!parent || !op)) return fail(c, PSG_EINVAL, "null parent / op");
  for (uint64_t i = 0; i < count; ++i) {
    if (op[i] > 2) return fail(c, PSG_EINVAL, "op must be 0 (copy), 1 (mutate) or 2 (fresh)");
    if (op[i] != 2 && parent[i] >= count) return fail(c, PSG_ERANGE, "parent index outside the population");
  }
  HIPCHK(c, hipSetDevice(c->cfg.device));
  HIPCHK(c, hipMemcpyAsync(c->d_parent, parent, sizeof(uint32_t) * count, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_op, op, count, hipMemcpyHostToDevice, c->stream));
  PopArgs a = pop_args(c, p, count);
  a.src = c->d_ho;
  a.ho = c->d_ho2;
  a.src_init = c->d_init;
  a.init = c->d_init2;
  a.parent = c->d_parent;
  a.op = c->d_op;
  HIPCHK(c, launch_population(a, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::swap(c->d_ho, c->d_ho2);  // the new generation is the loaded schedule / staged inputs
  std::swap(c->d_init, c->d_init2);
  std::swap(c->ho_cap, c->pop_cap);
  c->pop_cap = std::min(c->pop_cap, c->ho_cap);
  return PSG_OK;
}

int psg_population_read(psg_ctx* c, const uint32_t* rows, size_t k, uint64_t* ho, int32_t* init) {
  if (!c || (!rows && k) || (!ho && k)) return PSG_EINVAL;
  if (!c->subs.empty()) return fail(c, PSG_EINVAL, "device-resident populations need a single-device context");
  if (!c->ho_loaded) return fail(c, PSG_EINVAL, "no population loaded");
  HIPCHK(c, hipSetDevice(c->cfg.device));
  const uint64_t n = (uint64_t)c->cfg.n, R = (uint64_t)c->cfg.rounds, W = (uint64_t)c->W;
  for (size_t j = 0; j < k; ++j) {
    if (rows[j] >= c->ho_count) return fail(c, PSG_ERANGE, "row outside the population");
    HIPCHK(c, hipMemcpy(ho + j * R * n * W, c->d_ho + (uint64_t)rows[j] * R * n * W, sizeof(uint64_t) * R * n * W,
                        hipMemcpyDeviceToHost));
    if (init && c->staged)
      HIPCHK(c, hipMemcpy(init + j * n, c->d_init + (uint64_t)rows[j] * n, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  }
  return PSG_OK;
}

const char* psg_last_error(const psg_ctx* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

void psg_destroy(psg_ctx* c) {
  if (!c) return;
  if (!c->subs.empty() || c->cfg.n_devices > 0) {  // multi-device: the per-device contexts own everything
    for (psg_ctx* s : c->subs) psg_destroy(s);
    delete c;
    return;
  }
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_init) (void)hipFree(c->d_init);
  if (c->d_dec) (void)hipFree(c->d_dec);
  if (c->d_dround) (void)hipFree(c->d_dround);
  if (c->d_inst) (void)hipFree(c->d_inst);
  if (c->d_counters) (void)hipFree(c->d_counters);
  if (c->d_hand) (void)hipFree(c->d_hand);
  if (c->d_ids) (void)hipFree(c->d_ids);
  if (c->d_rec) (void)hipFree(c->d_rec);
  if (c->d_init_f64) (void)hipFree(c->d_init_f64);
  if (c->d_dec_f64) (void)hipFree(c->d_dec_f64);
  if (c->d_rec_f64) (void)hipFree(c->d_rec_f64);
  if (c->d_trace) (void)hipFree(c->d_trace);
  if (c->d_vm_counters) (void)hipFree(c->d_vm_counters);
  if (c->d_vm_err) (void)hipFree(c->d_vm_err);
  if (c->d_prog) (void)hipFree(c->d_prog);
  if (c->d_ho) (void)hipFree(c->d_ho);
  if (c->d_crash) (void)hipFree(c->d_crash);
  if (c->d_ho2) (void)hipFree(c->d_ho2);
  if (c->d_init2) (void)hipFree(c->d_init2);
  if (c->d_parent) (void)hipFree(c->d_parent);
  if (c->d_op) (void)hipFree(c->d_op);
  if (c->module) (void)hipModuleUnload(c->module);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

}  // extern "C"
