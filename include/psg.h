/*
 * psg.h — C ABI of the MI355X batched Heard-Of (HO) round executor and
 * Spec checker ("PSync GPU", psg).
 *
 * This is the drop-in boundary for ONE path of dzufferey/round (PSync): lockstep
 * execution of closed `Round`s over many independent consensus instances under
 * an HO schedule, with the algorithm's `Spec` evaluated after every round.
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference root; psync/ = src/main/scala/psync/, example/ = src/test/scala/example/):
 *
 *   psg_create          Algorithm construction + `Runtime.apply` backend choice
 *                       (psync/Algorithm.scala:13-31, psync/runtime/Runtime.scala:167-177)
 *                       and `RtProcess.setGroup` (psync/Process.scala:45-51): n, dense pids.
 *   psg_load_inputs     the per-process `ConsensusIO.initialValue` handed to
 *                       `Process.init(io)` (example/Otr.scala:21-26, LastVoting.scala:97-109, ...)
 *   psg_run_batch       `Algorithm.startInstance` for a range of instances
 *                       (psync/Algorithm.scala:36-42) followed by the whole
 *                       `InstanceHandler.run` round loop (psync/runtime/InstanceHandler.scala:164-258):
 *                       `init()` / `send` / `receive*` / `update` per round
 *                       (psync/Process.scala:67-82, psync/Round.scala:57-69, 102-124),
 *                       plus concrete evaluation of the `Spec` (psync/Specs.scala:8-16)
 *                       that the reference only checks symbolically
 *                       (psync/verification/Verifier.scala:111-275).
 *   psg_fetch_instances per-instance `ConsensusIO.decide` callbacks and final
 *                       process state for a sampled subset (the parity path).
 *   psg_last_error      `Logger.logAndThrow` messages (InstanceHandler.scala:346,351).
 *   psg_destroy         `Algorithm.stopInstance` / `Runtime.shutdown` (Runtime.scala:130-143).
 *
 * Conventions: every function returns 0 on success and a negative errno-style
 * code on failure (no exception, no abort crosses the ABI). The caller owns all
 * host buffers; the library owns device memory. A context is single-threaded.
 * It drives one HIP device (`device`) or, with `n_devices` > 0, the listed
 * devices: each call then splits its instance range into contiguous per-device
 * slices, runs them on one host thread per device and sums the summaries
 * (the reference's per-instance executor pool,
 * psync/runtime/Runtime.scala:43-57, 126-128). The other multi-GPU form is one
 * process per GPU, each with its own context over a shard of the global
 * instance-id range. Results are bit-identical for any split, because every
 * random draw is keyed on the global instance id.
 */
#ifndef PSG_H
#define PSG_H

#ifndef __HIPCC_RTC__ /* hiprtc builds of the kernel sources define the integer types */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define PSG_ABI_VERSION 4u

/* Algorithms, keyed on the reference class names. */
enum psg_alg {
  PSG_ALG_OTR = 1,         /* example.OTR            example/Otr.scala:13-128 */
  PSG_ALG_LAST_VOTING = 2, /* example.LastVoting     example/LastVoting.scala:11-212 */
  PSG_ALG_FLOODMIN = 3,    /* example.FloodMin       example/FloodMin.scala:8-48 */
  PSG_ALG_KSET = 4,        /* example.KSetAgreement  example/KSetAgreement.scala:21-87 */
  PSG_ALG_BENOR = 5,       /* example.BenOr          example/BenOr.scala:11-124 */
  /* second wave */
  PSG_ALG_OTR2 = 6,        /* example.OTR2               example/Otr2.scala:9-104 */
  PSG_ALG_SLV = 7,         /* example.ShortLastVoting    example/ShortLastVoting.scala:13-119 */
  PSG_ALG_KSET_ES = 8,     /* example.KSetEarlyStopping  example/KSetEarlyStopping.scala:9-57 */
  PSG_ALG_EPSILON = 9      /* example.EpsilonConsensus   example/Epsilon.scala:16-83 (Double values) */
};

/* Which element of a Scala immutable.Map is "first" (LastVoting maxBy ties,
 * LastVoting.scala:132; KSet find, KSetAgreement.scala:53). */
enum psg_tiebreak {
  PSG_TIE_CHAMP = 0,  /* Scala 2.13: insertion order (ascending pid) for <= 4 entries,
                         CHAMP hash-trie order for >= 5 entries (default) */
  PSG_TIE_MIN_PID = 1 /* always the smallest pid */
};

/* Error codes (negative errno values). */
#define PSG_OK 0
#define PSG_EINVAL (-22)
#define PSG_ENOMEM (-12)
#define PSG_ENODEV (-19)
#define PSG_EIO (-5)
#define PSG_ERANGE (-34)

#define PSG_MAX_N 256
#define PSG_MAX_ROUNDS 250
#define PSG_MAX_CHECKS 12
#define PSG_NEVER 0xFFu /* "never" marker in uint8 check-point fields */
#define PSG_MAX_DEVICES 16

/* Seeded adversarial HO schedule. All randomness is Philox4x32-10 keyed by
 * (seed_lo, seed_hi) with counter (inst_lo, inst_hi, round, pid | stream<<16);
 * see DESIGN.md "Schedule". Faults are HO sets (psync/Process.scala:14). */
typedef struct psg_schedule {
  uint32_t drop_log2;  /* 0: no benign loss; k>0: each non-self link lost w.p. 2^-k per round */
  uint32_t good_p32;   /* P(round is "good") * 2^32: every HO(p) = one common set s */
  int32_t good_min;    /* good-round common set satisfies |s| > good_min (<0: 2n/3, Otr.scala:96) */
  int32_t crash_fmax;  /* <0: no crash; else f ~ U{0..crash_fmax} processes crash (permanent
                          send omission from a crash round ~ U{0..R-1}; half the links
                          survive in the crash round) */
  int32_t ho_min;      /* <0: none; else if |HO(p)| <= ho_min then HO(p) := all
                          (BenOr safetyPredicate |HO(p)| > n/2, BenOr.scala:92) */
  uint32_t self_bit;   /* 1: p in HO(p) always (self send bypasses the network,
                          psync/Round.scala:114-116); 0: pure HO */
} psg_schedule;

typedef struct psg_config {
  uint32_t abi_version; /* must be PSG_ABI_VERSION */
  int32_t alg;          /* enum psg_alg */
  int32_t n;            /* processes per instance, 1..PSG_MAX_N */
  int32_t rounds;       /* R rounds executed per instance, 1..PSG_MAX_ROUNDS */
  uint64_t seed;
  int32_t value_range;  /* synthetic init values uniform in {1..value_range} (BenOr: {false,true};
                           EpsilonConsensus: Double uniform in [0,1) like Random.nextDouble, unused) */
  int32_t param;        /* OTR/OTR2 afterDecision (Otr.scala:89, default 2); FloodMin f (FloodMin.scala:27);
                           KSet k (KSetAgreement.scala:56); KSetEarlyStopping t; others unused */
  int32_t tiebreak;     /* enum psg_tiebreak */
  int32_t device;       /* HIP device ordinal (n_devices == 0) */
  int32_t variant;      /* 0 = reference algorithm; 1 = test mutation */
  uint64_t batch_capacity; /* max instances per psg_run_batch call (device buffers sized for it) */
  psg_schedule sched;
  int32_t param2;       /* KSetEarlyStopping k (KSetEarlyStopping.scala:9; param = t) */
  int32_t reserved;
  double real_param;    /* EpsilonConsensus epsilon (Epsilon.scala:16; param = f) */
  int32_t n_devices;    /* 0: the single device `device`; 1..PSG_MAX_DEVICES: run on devices[0..n_devices)
                           (an ordinal may repeat; batch_capacity is the whole context's, split evenly) */
  int32_t devices[PSG_MAX_DEVICES];
} psg_config;

/* Aggregate result of one batch. All fields are sums over instances (so a
 * cross-GPU all-reduce(sum) of the int64 array is the node-level result),
 * except kernel_ns. */
typedef struct psg_summary {
  int64_t instances;
  int64_t process_rounds;              /* checked process-rounds = n * R per instance (a
                                          halted process counts until its instance's last check) */
  int64_t active_process_rounds;       /* of those, rounds in which the process took a step (not yet
                                          halted at the round's start; psync/Round.scala:42-55) */
  int64_t live_instance_rounds;        /* instance-rounds with some process still active; the other
                                          n_rounds * instances - live ones evaluate the Spec only */
  int64_t fail_count[PSG_MAX_CHECKS];  /* instances in which check slot was false at some check point */
  int64_t decided_processes;           /* processes whose decide callback fired */
  int64_t digest;                      /* sum (mod 2^64) of per-instance digests */
  int64_t term_hist[PSG_MAX_ROUNDS + 2]; /* [c] = instances whose Termination first held at
                                            check point c (0..R); [R+1] = never */
  int64_t kernel_ns;                   /* device time of the round kernel (HIP events) */
} psg_summary;

/* Per-instance result (24 bytes). Check point c = number of completed rounds
 * (c = 0 is the initial state, c = R after the last round), i.e. the spec's r
 * (psync/verification/Verifier.scala:159-168, 237-243). */
typedef struct psg_instance_summary {
  uint64_t digest;                    /* hash of every process's (decision, decision round,
                                         halt round, final main variable) */
  uint8_t first_fail[PSG_MAX_CHECKS]; /* first check point where slot was false; PSG_NEVER */
  uint8_t term_round;                 /* first check point where all processes decided; PSG_NEVER */
  uint8_t n_checks;
  uint16_t n_decided;
} psg_instance_summary;

/* Per-process record (fetch path). For EpsilonConsensus (Double state) decision
 * and final_x hold fold32(bits) = low ^ high word of the IEEE-754 bits; the
 * values themselves come from the _f64 entry points below. */
typedef struct psg_process_record {
  int32_t decision;       /* value passed to ConsensusIO.decide (BenOr: 0/1); 0 if none */
  int32_t decision_round; /* round k (0-based) of the first decide callback, -1 if none */
  int32_t halt_round;     /* round k whose update called exitAtEndOfRound, -1 if never */
  int32_t final_x;        /* final main variable (OTR/LV/FloodMin x, BenOr x, KSet pick(t)) */
} psg_process_record;

/* ---------------------------------------------------------------------------
 * Generic Spec evaluation: a Spec given as a compiled
 * Formula program instead of the algorithm's hand-lowered checks.
 *
 * Replaces, for concrete checking, the Spec / Formula surface of the reference
 * (psync/Specs.scala:8-16, psync/formula/Formula.scala: ForAll / Exists /
 * Comprehension / Cardinality / Literal / Variable / Application; the `init` /
 * `old` wrappers and Option isDefined / get of psync/macros/FormulaExtractor.scala).
 * The host compiler (round_amd/formula.py) turns a Formula tree into this
 * stack bytecode; the device evaluates it after every round over a trace of the
 * process states. Quantified process variables range over the pids 0..n-1,
 * V.exists over Int is finitized exactly (candidate values compared with the
 * variable, +-1, plus Int.MinValue / Int.MaxValue).
 * ------------------------------------------------------------------------- */

/* Process-state fields visible to a Spec (the variables the reference specs read). */
enum psg_field {
  PSG_FIELD_X = 0,        /* x (OTR/LV/FloodMin/SLV), est (KSetEarlyStopping), pick(t) (KSet), x (BenOr 0/1) */
  PSG_FIELD_DECIDED = 1,  /* decided flag (ghost for algorithms without one: decide callback fired) */
  PSG_FIELD_DECISION = 2, /* decision (OTR2: Option, PSG_NONE32 when empty) */
  PSG_FIELD_TS = 3,       /* LastVoting / ShortLastVoting ts */
  PSG_FIELD_READY = 4,    /* LastVoting ready */
  PSG_FIELD_COMMIT = 5,   /* LastVoting / ShortLastVoting commit */
  PSG_FIELD_VOTE = 6,     /* LastVoting / SLV vote; BenOr vote (Option[Boolean], PSG_NONE32 when empty) */
  PSG_FIELD_CANDECIDE = 7,/* BenOr canDecide */
  PSG_FIELD_HOSIZE = 8,   /* |mailbox| of the round just executed (n if the process took no step) */
  PSG_NFIELDS = 9
};
/* Which state a field is read from (FormulaExtractor init(...) / old(...)). */
enum psg_tag { PSG_TAG_CUR = 0, PSG_TAG_OLD = 1, PSG_TAG_INIT = 2 };
#define PSG_NONE32 ((int32_t)0x80000000) /* Option None in an int32 field */

/* Bytecode: word = op | a << 8 | b << 16 (b signed 16-bit). Per-lane int32 stack. */
enum psg_op {
  PSG_OP_HALT = 0,   /* end of an expression: result = top of stack */
  PSG_OP_IMM = 1,    /* push b */
  PSG_OP_IMM32 = 2,  /* push the next code word */
  PSG_OP_N = 3,      /* push n */
  PSG_OP_R = 4,      /* push r (check point: completed rounds) */
  PSG_OP_VAR = 5,    /* push bound variable a */
  PSG_OP_FIELD = 6,  /* p = pop; push field a (enum psg_field) of process p in state b (enum psg_tag) */
  PSG_OP_NOT = 7, PSG_OP_NEG = 8, PSG_OP_ISDEF = 9, /* ISDEF: v != PSG_NONE32 */
  PSG_OP_AND = 10, PSG_OP_OR = 11, PSG_OP_IMPL = 12,
  PSG_OP_EQ = 13, PSG_OP_NE = 14, PSG_OP_LT = 15, PSG_OP_LE = 16, PSG_OP_GT = 17, PSG_OP_GE = 18,
  PSG_OP_ADD = 19, PSG_OP_SUB = 20, PSG_OP_MUL = 21,
  PSG_OP_DIV = 22, PSG_OP_MOD = 23, /* Scala Int semantics (truncation); x / 0 and x % 0 evaluate to 0 */
  PSG_OP_BIND = 24,  /* bound variable a = pop (Set.contains(e) of a comprehension) */
  PSG_OP_QBEGIN = 25,/* quantifier kind a over bound variable b; next word: pc of the matching QEND;
                        EXISTS_VI: then one word = (#expression candidates popped from the stack) | (#field
                        sets) << 16, then one word per field set = field | tag << 8 */
  PSG_OP_QEND = 26,
  PSG_OP_COORD = 27  /* push (r / 4) % n (LastVoting / ShortLastVoting coord(r/4)) */
};
enum psg_quant {
  PSG_Q_FORALL_P = 0, PSG_Q_EXISTS_P = 1, PSG_Q_COUNT_P = 2,    /* over pids, one at a time */
  PSG_Q_FORALL_PL = 3, PSG_Q_EXISTS_PL = 4, PSG_Q_COUNT_PL = 5, /* over pids, one lane per pid (not nested) */
  PSG_Q_EXISTS_VB = 6,                                          /* V.exists over Boolean */
  PSG_Q_EXISTS_VI = 7                                           /* V.exists over Int (finitized) */
};
#define PSG_SPEC_RELATIONAL 1 /* slot flag: reads old(...), vacuously true at check point 0 */

typedef struct psg_spec_program {
  int32_t n_slots;           /* check slots, 1..PSG_MAX_CHECKS */
  int32_t n_words;           /* code length */
  const int32_t* code;       /* bytecode */
  const int32_t* slot_entry; /* [n_slots] pc of each slot's expression (ends in PSG_OP_HALT) */
  const int32_t* slot_flags; /* [n_slots] PSG_SPEC_* */
  int32_t term_entry;        /* pc of the Termination expression, -1 for none */
  int32_t n_vars;            /* bound variables used, <= 16 */
  const char* module_path;   /* NULL: interpret the bytecode; else a gfx950 code object with kernels
                                psg_spec_native_w1..w4 (the same Spec lowered to wave code by
                                round_amd/formula.py compile_native), launched instead; a fused module
                                also holds psg_fused_a<alg>_w<W> / psg_fused_x_a<alg>_w<W> and records
                                its algorithm in the device global `psg_spec_alg` */
  int32_t alg;               /* 0: not bound to an algorithm; else the enum psg_alg the program was
                                compiled for (a mismatch with the context is PSG_EINVAL) */
} psg_spec_program;

typedef struct psg_ctx psg_ctx;

/* Fill *cfg with the defaults for algorithm alg at n processes. */
int psg_config_default(psg_config* cfg, int32_t alg, int32_t n);

/* Number of check slots of an algorithm and their names ("Safety", "Agreement", ...). */
int psg_check_count(int32_t alg);
const char* psg_check_name(int32_t alg, int32_t slot);

/* Map a reference class name ("example.OTR", "example.LastVoting", ...) to an alg id. */
int psg_alg_from_class(const char* class_name);

int psg_create(psg_ctx** out, const psg_config* cfg);

/* Stage the initial values of instances [inst_begin, inst_begin+inst_count) in
 * HBM, layout [instance][pid] int32. host_init == NULL: seeded synthetic values
 * generated on the device. A later psg_run_batch over exactly this range reads
 * them; any other range regenerates seeded values first (outside kernel_ns). */
int psg_load_inputs(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count,
                    const int32_t* host_init);

/* Execute R rounds of instances [inst_begin, inst_begin+inst_count) and evaluate
 * the Spec after every round. per_inst (nullable) receives inst_count
 * per-instance summaries. Blocks until the results are on the host. */
int psg_run_batch(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count,
                  psg_summary* out, psg_instance_summary* per_inst);

/* Copy the per-process decide results of the last batch: decision [count][n]
 * int32 and decision_round [count][n] int32 (-1 = none). Either may be NULL. */
int psg_copy_decisions(psg_ctx* ctx, int32_t* decision, int32_t* decision_round);

/* The instance count of the last batch (psg_run_batch / psg_run_batch_spec, 0 after an
 * empty one): the [count][n] size psg_copy_decisions writes. The library's own record, so
 * a binding sizing host arrays (the JNI shim) never trusts a copy of its own. */
int psg_last_batch_count(const psg_ctx* ctx, uint64_t* count);

/* Re-execute the listed global instance ids and return their summaries (k
 * entries) and per-process records (k * n entries, nullable). Inputs: the staged
 * ones (psg_load_inputs) when every id lies in the staged range, else seeded;
 * HO sets: the loaded explicit schedule (every id must lie in its range) or seeded. */
int psg_fetch_instances(psg_ctx* ctx, const uint64_t* ids, size_t k,
                        psg_instance_summary* sums, psg_process_record* procs);

/* Like psg_run_batch, but the Spec is the given program: fail_count / term_hist /
 * first_fail / term_round come from it (digest, decisions, records from the
 * round execution as usual). Integer-state algorithms only (not EpsilonConsensus).
 * The process states of every check point are traced in HBM and evaluated by the
 * device interpreter; large batches are processed in chunks of at most
 * PSG_SPEC_TRACE_MB (environment, default 2048) MiB of trace. */
int psg_run_batch_spec(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count, const psg_spec_program* prog,
                       psg_summary* out, psg_instance_summary* per_inst);

/* Compile a Spec given as Formula text — the S-expression form of the reference's own
 * Formula trees (psync/formula/Formula.scala: Binding ForAll / Exists / Comprehension,
 * Application, Variable, Literal), as integration/scala/GpuSpec.scala writes it from a
 * psync.Spec; format in round_amd/formula.py ("Formula text") — into *out for
 * psg_run_batch_spec. Replaces, for concrete checking, the Verifier's assembly of the
 * Spec (psync/verification/Verifier.scala:111-141). Host code, no device needed.
 * alg (enum psg_alg, 0 = unchecked) restricts the fields to the algorithm's state and is
 * recorded in out->alg. The arrays are the library's: release them with psg_spec_release.
 * names (nullable) receives the slot names, '\n'-separated ("Safety", "Invariant0", ...,
 * the property names, "SafetyPredicate"); PSG_ERANGE (nothing allocated) when names_len is
 * too small for all of them, err then says how many bytes are needed. Text nested deeper
 * than 512 forms is refused (PSG_EINVAL). err (nullable) the reason of a failure. */
int psg_spec_from_text(const char* text, int32_t alg, psg_spec_program* out, char* names, size_t names_len,
                       char* err, size_t err_len);
void psg_spec_release(psg_spec_program* prog);

/* Native lowering of Formula text, in-process (the C-ABI / JVM route to what
 * round_amd/formula.py compile_native builds from Python; replaces, for concrete checking, the
 * Verifier's lowering of a psync.Spec, psync/Specs.scala:8-16, psync/formula/Formula.scala:5-585).
 * The program is psg_spec_from_text's; out->module_path names a gfx950 code object generated
 * from the same Formula tree (equality pins, count guards, breakpoint finitization, tuple
 * quantifiers, memoized init membership, hoisted common subformulas) and compiled with hiprtc,
 * cached by a hash of its source and the kernel headers in cache_dir (NULL: <library
 * dir>/../build/spec, shared with formula.compile_native). fused != 0: the module also holds
 * the algorithm's round kernel with the Spec as its check hook, so psg_run_batch_spec runs one
 * launch; n > 0 limits its instantiations to that group size. The path string is the library's
 * (valid until the process exits); release the arrays with psg_spec_release. Kernel sources
 * are read from <library dir>/csrc and <library dir>/../include (PSG_CSRC / PSG_INCLUDE
 * override). No device needed to compile. */
int psg_spec_compile_native(const char* text, int32_t alg, int32_t fused, int32_t n, const char* cache_dir,
                            psg_spec_program* out, char* names, size_t names_len, char* err, size_t err_len);
/* The Spec of Formula text after the native lowering's exact V.exists / quantifier rewrites
 * (hoisted conjuncts free of a bound variable, split foralls), as Formula text — invariants
 * already guarded by their round invariants, (phase 1) — so the rewrites can be checked
 * against the Spec as written under any evaluator (tests). Same buffer contract as
 * psg_spec_native_source. Generator options for all three entry points (comma-separated:
 * nosym, sym — the symmetric-check-point lowering off / on; fused LastVoting modules default to
 * off —, nosplit, nofrozen, D<NAME>=<VALUE>) come from psg_spec_set_options on the calling thread, else
 * from the environment variable PSG_SPEC_OPTIONS; an unknown option, a define outside the
 * generator knobs (PSG_PHASE_TIMERS, the PSG_*_WPE occupancy targets and the exact-alternative
 * switches PSG_PHILOX_OPAQUE_KEYS, PSG_PHILOX_MAD64, PSG_XSHFL_MASK, PSG_QUEUE_CHUNK[_WIDE|_LANE],
 * PSG_MAJ_BITVOTE, PSG_BO_FLAGS_DPP) or a non-integer value makes the entry point return
 * PSG_EINVAL. */
int psg_spec_rewrite_text(const char* text, int32_t alg, char* out, size_t* out_len, char* err, size_t err_len);
/* The HIP source psg_spec_compile_native compiles for these arguments (tests, inspection):
 * *src_len = capacity in, the size needed (with the terminating NUL) out; PSG_ERANGE when
 * src is NULL or too small. */
int psg_spec_native_source(const char* text, int32_t alg, int32_t fused, int32_t n, char* src, size_t* src_len,
                           char* err, size_t err_len);
/* The generator options of the CALLING THREAD for the three entry points above (thread-local:
 * concurrent callers with different options never see each other's); NULL = back to the
 * environment's PSG_SPEC_OPTIONS. PSG_EINVAL (and nothing changed) for an invalid string. */
int psg_spec_set_options(const char* options);

/* Real-valued algorithms (PSG_ALG_EPSILON, RealConsensusIO, Epsilon.scala:10-13).
 * Same contracts as the int32 entry points; other algorithms get PSG_EINVAL.
 * host_init: [count][n] Double initial values, NULL = seeded (uniform [0,1)). */
int psg_load_inputs_f64(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count, const double* host_init);
/* decision [count][n] (0.0 if none) and decision_round [count][n] of the last batch. */
int psg_copy_decisions_f64(psg_ctx* ctx, double* decision, int32_t* decision_round);
/* psg_fetch_instances plus the Double decision and final x of each process ([k][n] each, nullable). */
int psg_fetch_instances_f64(psg_ctx* ctx, const uint64_t* ids, size_t k, psg_instance_summary* sums,
                            psg_process_record* procs, double* decision, double* final_x);

/* ---------------------------------------------------------------------------
 * Explicit HO schedules (replayable counterexamples and the
 * adversary search; the in-JVM harness of §8c driven by identical HO sets).
 *
 * In the reference an HO set is whatever the network delivered before the
 * round's timeout (psync/Round.scala:57-69, psync/runtime/InstanceHandler.scala:
 * 164-258); `Process.HO` is its Spec-level name (psync/Process.scala:14). Here it
 * is data: ho[inst][k][p] = HO(p) in round k as W = ceil(n/64) little-endian
 * 64-bit words (bit q of word w = process 64w+q), layout [count][R][n][W] uint64.
 * Sets are used verbatim (no self bit, no ho_min, no good rounds; bits >= n are
 * ignored). crash_round [count][n] (nullable: every process correct) only marks
 * processes as crashed for the checks that quantify over correct processes
 * (FloodMin / KSet k-agreement); the omissions themselves are in the HO sets.
 * ------------------------------------------------------------------------- */

/* Stage an explicit schedule for instances [inst_begin, inst_begin+inst_count)
 * (count <= batch_capacity). Until psg_clear_schedule, psg_run_batch,
 * psg_run_batch_spec and psg_fetch_instances read HO sets from it and accept only
 * instances inside its range (PSG_ERANGE otherwise). Initial values still come
 * from psg_load_inputs (or are seeded); BenOr coins stay seeded by instance id. */
int psg_load_schedule(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count, const uint64_t* ho,
                      const int32_t* crash_round);
/* Return to seeded HO schedules. */
int psg_clear_schedule(psg_ctx* ctx);
/* Export the seeded schedule of instances [inst_begin, inst_begin+inst_count)
 * in the explicit layout: ho [count][R][n][W] and crash_round [count][n] (-1 =
 * correct; nullable). Replaying it with psg_load_schedule reproduces the seeded
 * run bit for bit. Any count (processed in device chunks). */
int psg_materialize_schedule(psg_ctx* ctx, uint64_t inst_begin, uint64_t inst_count, uint64_t* ho,
                             int32_t* crash_round);

/* Device-resident search populations: the adversary search's generate /
 * mutate step (round_amd/adversary.py) on the GPU, so HO sets never cross PCIe.
 * A population is the loaded explicit schedule + the staged initial values of
 * [inst_begin, inst_begin+count); general-omission fault model (every link of
 * every round independently present or not). All draws are Philox4x32-10 keyed
 * by `seed` with the generation number in the counter, so a population is a
 * pure function of its parameters. */
typedef struct psg_population_params {
  uint64_t seed;            /* generator key */
  uint32_t generation;      /* distinct draws per generation */
  uint32_t flips;           /* links (k, p, q) flipped per mutant (q != p when self_bit) */
  int32_t min_size;         /* repair: |HO(p)| >= min_size after generation / mutation (<= 0: none);
                               BenOr safetyPredicate |HO(p)| > n/2 (BenOr.scala:92) = n/2 + 1 */
  uint32_t self_bit;        /* p in HO(p) (psync/Round.scala:114-116) */
  uint32_t keep_p256[4];    /* fresh schedules: each link present w.p. keep/256; schedule i uses level i % 4 */
  int32_t value_range;      /* initial values uniform in {1..value_range} (BenOr: {0, 1}) */
  uint32_t redraw_p256;     /* a mutant redraws each initial value w.p. redraw/256 */
} psg_population_params;

/* Fresh random population over [inst_begin, inst_begin+count) (count <= batch_capacity);
 * afterwards the range is loaded exactly as by psg_load_schedule + psg_load_inputs. */
int psg_population_fresh(psg_ctx* ctx, uint64_t inst_begin, uint64_t count, const psg_population_params* p);
/* Next generation, in place over the loaded population: slot i becomes op[i] == 0 a copy of
 * slot parent[i], 1 a mutant of slot parent[i] (flips + redraws, then repair), 2 a fresh
 * schedule (count entries each; parents index the current population). */
int psg_population_next(psg_ctx* ctx, const uint32_t* parent, const uint8_t* op, const psg_population_params* p);
/* Copy slots rows[0..k) of the loaded population to the host: ho [k][R][n][W], init [k][n] (nullable). */
int psg_population_read(psg_ctx* ctx, const uint32_t* rows, size_t k, uint64_t* ho, int32_t* init);

const char* psg_last_error(const psg_ctx* ctx);
void psg_destroy(psg_ctx* ctx);

/* Library-level error text when psg_create itself fails (ctx unavailable). */
const char* psg_create_error(void);

/* Self-test hook (tests only, no reference counterpart): for each of `count` pid
 * sets given as 64-bit masks (pids < 64), the first pid in Scala Map iteration
 * order (enum psg_tiebreak), computed on device `device` by the helper that
 * resolves a per-receiver `mailbox.head` (ShortLastVoting.scala:87). -1 for an
 * empty set. */
int psg_selftest_map_head(int32_t device, const uint64_t* sets, int32_t count, int32_t tiebreak, int32_t* out_first);

/* Self-test hook (tests only): runs `n_ops` (opcode, pos) pairs on one W-word HO mask
 * (Mask<W>, W = 1..4) on device `device`, the device analogue of psync.utils.LongBitSet
 * (LongBitSet.scala:5-33: a 64-bit set whose index is taken mod 64; W words: mod 64W).
 * Opcodes: 0 empty, 1 full, 2 set(pos), 3 clear(pos), 4 flip(pos), 5 get(pos) -> out,
 * 6 size -> out. Results of get / size are written to out[0..n_out) in order. */
int psg_selftest_bitset(int32_t device, int32_t W, const int32_t* ops, int32_t n_ops, int32_t* out, int32_t n_out);

#ifdef __cplusplus
}
#endif

#endif /* PSG_H */
