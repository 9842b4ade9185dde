/*
 * psg_jni.c — JNI binding of include/psg.h for the Scala `psync.gpu.GpuRound`
 * plugin (integration/scala/GpuRound.scala).
 *
 * Build on a machine with a JDK:
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" \
 *       -I<repo>/include psg_jni.c -L<repo>/round_amd -lpsg -Wl,-rpath,<repo>/round_amd \
 *       -o libpsg_jni.so
 * and load it with System.loadLibrary("psg_jni"). In this repository (no JDK) the
 * file is compiled against integration/jni/jni_min/jni.h, a declaration-only
 * subset of the JNI types and functions it calls (tests/test_jni_shim.py), so the
 * signatures, JNI name mangling and argument checks are compile-checked on every run.
 *
 * Each native method maps onto a C-ABI entry point; errors become
 * java.lang.IllegalStateException / IllegalArgumentException carrying
 * psg_last_error(), mirroring the reference's Logger.logAndThrow
 * (psync/runtime/InstanceHandler.scala:346, 351). Every Java array is checked
 * against the cell count the C ABI will read or write before its elements are
 * taken, so a short array throws IllegalArgumentException instead of being read
 * or written past its end.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "psg.h"

/* The Java handle: the context plus the shape the array checks need. */
typedef struct jctx {
  psg_ctx* ctx;
  int64_t n, rounds, words; /* words = ceil(n / 64) */
} jctx;

static void throw_cls(JNIEnv* env, const char* cls, const char* msg) {
  jclass ex = (*env)->FindClass(env, cls);
  if (ex) (*env)->ThrowNew(env, ex, msg);
}

static void throw_psg(JNIEnv* env, int rc, const char* msg) {
  char buf[512];
  snprintf(buf, sizeof buf, "psg error %d: %s", rc, msg ? msg : "");
  throw_cls(env, rc == PSG_EINVAL || rc == PSG_ERANGE ? "java/lang/IllegalArgumentException"
                                                       : "java/lang/IllegalStateException", buf);
}

/* 1 if `arr` holds at least `need` elements (need >= 0), else throws and returns 0.
 * A null array is accepted only when `nullable`. */
static int check_len(JNIEnv* env, jarray arr, int64_t need, int nullable, const char* what) {
  char buf[256];
  if (!arr) {
    if (nullable) return 1;
    snprintf(buf, sizeof buf, "%s must not be null", what);
    throw_cls(env, "java/lang/IllegalArgumentException", buf);
    return 0;
  }
  const int64_t have = (int64_t)(*env)->GetArrayLength(env, arr);
  if (need < 0 || have < need) {
    snprintf(buf, sizeof buf, "%s has %lld elements, %lld needed", what, (long long)have, (long long)need);
    throw_cls(env, "java/lang/IllegalArgumentException", buf);
    return 0;
  }
  return 1;
}

/* Cells of the last batch's [count][n] decision arrays, from the library's own record
 * (psg_last_batch_count): an empty batch after a large one yields 0, never a stale size. */
static int64_t last_cells(const jctx* j) {
  uint64_t count = 0;
  if (psg_last_batch_count(j->ctx, &count)) return 0;
  return (int64_t)count * j->n;
}

static jctx* J(JNIEnv* env, jlong h) {
  jctx* j = (jctx*)(intptr_t)h;
  if (!j) throw_cls(env, "java/lang/IllegalStateException", "GpuRound context is closed");
  return j;
}

static int count_ok(JNIEnv* env, jlong begin, jlong count) {
  if (begin < 0 || count < 0) {
    throw_cls(env, "java/lang/IllegalArgumentException", "begin / count must be >= 0");
    return 0;
  }
  return 1;
}

/* long create(int alg, int n, int rounds, long seed, int valueRange, int param, int param2, double realParam,
 *             int tiebreak, int device, int variant, long batchCapacity,
 *             int dropLog2, int goodP32, int goodMin, int crashFmax, int hoMin, boolean selfBit,
 *             int[] devicesOrNull)
 * devices: run every batch split over these HIP devices, one host thread each (psg_config.n_devices). */
JNIEXPORT jlong JNICALL Java_psync_gpu_GpuRoundNative_00024_create(
    JNIEnv* env, jobject self, jint alg, jint n, jint rounds, jlong seed, jint valueRange, jint param, jint param2,
    jdouble realParam, jint tiebreak, jint device, jint variant, jlong batchCapacity, jint dropLog2, jint goodP32,
    jint goodMin, jint crashFmax, jint hoMin, jboolean selfBit, jintArray devices) {
  (void)self;
  psg_config c;
  memset(&c, 0, sizeof c);
  c.abi_version = PSG_ABI_VERSION;
  c.alg = alg;
  c.n = n;
  c.rounds = rounds;
  c.seed = (uint64_t)seed;
  c.value_range = valueRange;
  c.param = param;
  c.param2 = param2;
  c.real_param = realParam;
  c.tiebreak = tiebreak;
  c.device = device;
  c.variant = variant;
  c.batch_capacity = (uint64_t)batchCapacity;
  c.sched.drop_log2 = (uint32_t)dropLog2;
  c.sched.good_p32 = (uint32_t)goodP32;
  c.sched.good_min = goodMin;
  c.sched.crash_fmax = crashFmax;
  c.sched.ho_min = hoMin;
  c.sched.self_bit = selfBit ? 1u : 0u;
  if (devices) {
    const jsize k = (*env)->GetArrayLength(env, devices);
    if (k < 1 || k > PSG_MAX_DEVICES) {
      throw_cls(env, "java/lang/IllegalArgumentException", "devices must list 1..16 HIP devices");
      return 0;
    }
    (*env)->GetIntArrayRegion(env, devices, 0, k, (jint*)c.devices);
    c.n_devices = k;
  }
  jctx* j = (jctx*)calloc(1, sizeof(jctx));
  if (!j) {
    throw_psg(env, PSG_ENOMEM, "out of host memory");
    return 0;
  }
  int rc = psg_create(&j->ctx, &c);
  if (rc) {
    free(j);
    throw_psg(env, rc, psg_create_error());
    return 0;
  }
  j->n = n;
  j->rounds = rounds;
  j->words = (n + 63) / 64;
  return (jlong)(intptr_t)j;
}

/* void loadInputs(long ctx, long begin, long count, int[] init) — init may be null (seeded) */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadInputs(JNIEnv* env, jobject self, jlong h,
                                                                      jlong begin, jlong count, jintArray init) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) || !check_len(env, init, count * j->n, 1, "init")) return;
  jint* p = init ? (*env)->GetIntArrayElements(env, init, NULL) : NULL;
  int rc = psg_load_inputs(j->ctx, (uint64_t)begin, (uint64_t)count, (const int32_t*)p);
  if (p) (*env)->ReleaseIntArrayElements(env, init, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

static jlongArray summary_array(JNIEnv* env, const psg_summary* s) {
  const jsize len = (jsize)(sizeof(psg_summary) / sizeof(int64_t));
  jlongArray out = (*env)->NewLongArray(env, len);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, len, (const jlong*)s);
  return out;
}

/* long[] runBatch(long ctx, long begin, long count, byte[] perInstanceOrNull)
 * returns the psg_summary as a flat long[] (struct order); perInstance receives
 * count * sizeof(psg_instance_summary) bytes when non-null. */
JNIEXPORT jlongArray JNICALL Java_psync_gpu_GpuRoundNative_00024_runBatch(JNIEnv* env, jobject self, jlong h,
                                                                          jlong begin, jlong count,
                                                                          jbyteArray perInst) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) ||
      !check_len(env, perInst, count * (int64_t)sizeof(psg_instance_summary), 1, "perInstance"))
    return NULL;
  psg_summary s;
  psg_instance_summary* pi = NULL;
  if (perInst && count) {
    pi = (psg_instance_summary*)malloc(sizeof(psg_instance_summary) * (size_t)count);
    if (!pi) {
      throw_psg(env, PSG_ENOMEM, "out of host memory");
      return NULL;
    }
  }
  int rc = psg_run_batch(j->ctx, (uint64_t)begin, (uint64_t)count, &s, pi);
  if (rc) {
    free(pi);
    throw_psg(env, rc, psg_last_error(j->ctx));
    return NULL;
  }
  if (pi) {
    (*env)->SetByteArrayRegion(env, perInst, 0, (jsize)(sizeof(psg_instance_summary) * (size_t)count),
                               (const jbyte*)pi);
    free(pi);
  }
  return summary_array(env, &s);
}

/* long[] runBatchSpec(long ctx, long begin, long count, int[] code, int[] slotEntry, int[] slotFlags,
 *                     int termEntry, int nVars, int alg, String modulePathOrNull, byte[] perInstanceOrNull)
 * psg_run_batch_spec: the Spec is a compiled psg_spec_program (GpuSpec.compile, integration/scala/
 * GpuSpec.scala) instead of the algorithm's built-in checks. */
JNIEXPORT jlongArray JNICALL Java_psync_gpu_GpuRoundNative_00024_runBatchSpec(
    JNIEnv* env, jobject self, jlong h, jlong begin, jlong count, jintArray code, jintArray slotEntry,
    jintArray slotFlags, jint termEntry, jint nVars, jint alg, jstring modulePath, jbyteArray perInst) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) || !check_len(env, code, 1, 0, "code") ||
      !check_len(env, slotEntry, 1, 0, "slotEntry") ||
      !check_len(env, perInst, count * (int64_t)sizeof(psg_instance_summary), 1, "perInstance"))
    return NULL;
  const jsize nslots = (*env)->GetArrayLength(env, slotEntry);
  if (!check_len(env, slotFlags, nslots, 0, "slotFlags")) return NULL;
  psg_spec_program p;
  memset(&p, 0, sizeof p);
  p.n_slots = nslots;
  p.n_words = (*env)->GetArrayLength(env, code);
  p.term_entry = termEntry;
  p.n_vars = nVars;
  p.alg = alg;
  jint* cd = (*env)->GetIntArrayElements(env, code, NULL);
  jint* se = (*env)->GetIntArrayElements(env, slotEntry, NULL);
  jint* sf = (*env)->GetIntArrayElements(env, slotFlags, NULL);
  const char* mp = modulePath ? (*env)->GetStringUTFChars(env, modulePath, NULL) : NULL;
  p.code = (const int32_t*)cd;
  p.slot_entry = (const int32_t*)se;
  p.slot_flags = (const int32_t*)sf;
  p.module_path = mp;
  psg_summary s;
  psg_instance_summary* pi = NULL;
  int rc = PSG_OK;
  if (perInst && count) {
    pi = (psg_instance_summary*)malloc(sizeof(psg_instance_summary) * (size_t)count);
    if (!pi) rc = PSG_ENOMEM;
  }
  if (rc == PSG_OK) rc = psg_run_batch_spec(j->ctx, (uint64_t)begin, (uint64_t)count, &p, &s, pi);
  if (mp) (*env)->ReleaseStringUTFChars(env, modulePath, mp);
  (*env)->ReleaseIntArrayElements(env, code, cd, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, slotEntry, se, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, slotFlags, sf, JNI_ABORT);
  if (rc) {
    free(pi);
    throw_psg(env, rc, rc == PSG_ENOMEM ? "out of host memory" : psg_last_error(j->ctx));
    return NULL;
  }
  if (pi) {
    (*env)->SetByteArrayRegion(env, perInst, 0, (jsize)(sizeof(psg_instance_summary) * (size_t)count),
                               (const jbyte*)pi);
    free(pi);
  }
  return summary_array(env, &s);
}

/* int[] compileSpec(String text, int alg) — psg_spec_from_text: the Formula text of a Spec
 * (integration/scala/GpuSpec.scala) compiled to bytecode, returned packed as
 * [nSlots, nWords, termEntry, nVars, code[nWords], slotEntry[nSlots], slotFlags[nSlots]]. */
JNIEXPORT jintArray JNICALL Java_psync_gpu_GpuRoundNative_00024_compileSpec(JNIEnv* env, jobject self, jstring text,
                                                                            jint alg) {
  (void)self;
  if (!text) {
    throw_cls(env, "java/lang/IllegalArgumentException", "text must not be null");
    return NULL;
  }
  const char* t = (*env)->GetStringUTFChars(env, text, NULL);
  psg_spec_program p;
  char err[512];
  const int rc = psg_spec_from_text(t, alg, &p, NULL, 0, err, sizeof err);
  (*env)->ReleaseStringUTFChars(env, text, t);
  if (rc) {
    throw_psg(env, rc, err);
    return NULL;
  }
  const jsize len = 4 + p.n_words + 2 * p.n_slots;
  jintArray out = (*env)->NewIntArray(env, len);
  if (out) {
    const jint head[4] = {p.n_slots, p.n_words, p.term_entry, p.n_vars};
    (*env)->SetIntArrayRegion(env, out, 0, 4, head);
    (*env)->SetIntArrayRegion(env, out, 4, p.n_words, (const jint*)p.code);
    (*env)->SetIntArrayRegion(env, out, 4 + p.n_words, p.n_slots, (const jint*)p.slot_entry);
    (*env)->SetIntArrayRegion(env, out, 4 + p.n_words + p.n_slots, p.n_slots, (const jint*)p.slot_flags);
  }
  psg_spec_release(&p);
  return out;
}

/* String compileSpecNames(String text, int alg) — the slot names of compileSpec's program,
 * '\n'-separated ("Safety", "Invariant0", ..., property names, "SafetyPredicate"). */
JNIEXPORT jstring JNICALL Java_psync_gpu_GpuRoundNative_00024_compileSpecNames(JNIEnv* env, jobject self,
                                                                               jstring text, jint alg) {
  (void)self;
  if (!text) {
    throw_cls(env, "java/lang/IllegalArgumentException", "text must not be null");
    return NULL;
  }
  const char* t = (*env)->GetStringUTFChars(env, text, NULL);
  psg_spec_program p;
  char err[512];
  /* PSG_ERANGE = the buffer cannot hold every slot name: grow it, never truncate (the
   * names must line up with compileSpec's slotEntry / slotFlags) */
  size_t len = 4096;
  char* names = NULL;
  int rc = PSG_ERANGE;
  while (rc == PSG_ERANGE && len <= ((size_t)1 << 24)) {
    char* grown = (char*)realloc(names, len);
    if (!grown) {
      rc = PSG_ENOMEM;
      snprintf(err, sizeof err, "out of host memory");
      break;
    }
    names = grown;
    rc = psg_spec_from_text(t, alg, &p, names, len, err, sizeof err);
    len *= 2;
  }
  (*env)->ReleaseStringUTFChars(env, text, t);
  if (rc) {
    free(names);
    throw_psg(env, rc, err);
    return NULL;
  }
  psg_spec_release(&p);
  jstring out = (*env)->NewStringUTF(env, names);
  free(names);
  return out;
}

/* String compileSpecNative(String text, int alg, boolean fused, int n) — psg_spec_compile_native:
 * the Spec's Formula text lowered to gfx950 code in the library (hiprtc, cached; fused: with the
 * algorithm's round kernel), returned as the code object's path for runBatchSpec's modulePath
 * (the program itself is compileSpec's). */
JNIEXPORT jstring JNICALL Java_psync_gpu_GpuRoundNative_00024_compileSpecNative(JNIEnv* env, jobject self,
                                                                                jstring text, jint alg,
                                                                                jboolean fused, jint n) {
  (void)self;
  if (!text) {
    throw_cls(env, "java/lang/IllegalArgumentException", "text must not be null");
    return NULL;
  }
  const char* t = (*env)->GetStringUTFChars(env, text, NULL);
  psg_spec_program p;
  char err[4096];
  const int rc = psg_spec_compile_native(t, alg, fused ? 1 : 0, n, NULL, &p, NULL, 0, err, sizeof err);
  (*env)->ReleaseStringUTFChars(env, text, t);
  if (rc) {
    throw_psg(env, rc, err);
    return NULL;
  }
  jstring out = (*env)->NewStringUTF(env, p.module_path);
  psg_spec_release(&p);
  return out;
}

/* void copyDecisions(long ctx, int[] decision, int[] decisionRound) — the batched
 * ConsensusIO.decide results of the last batch, [count][n] each (either may be null). */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_copyDecisions(JNIEnv* env, jobject self, jlong h,
                                                                         jintArray dec, jintArray drnd) {
  (void)self;
  jctx* j = J(env, h);
  const int64_t cells = j ? last_cells(j) : 0;
  if (!j || !check_len(env, dec, cells, 1, "decision") || !check_len(env, drnd, cells, 1, "decisionRound")) return;
  jint* d = dec ? (*env)->GetIntArrayElements(env, dec, NULL) : NULL;
  jint* r = drnd ? (*env)->GetIntArrayElements(env, drnd, NULL) : NULL;
  int rc = psg_copy_decisions(j->ctx, (int32_t*)d, (int32_t*)r);
  if (d) (*env)->ReleaseIntArrayElements(env, dec, d, 0);
  if (r) (*env)->ReleaseIntArrayElements(env, drnd, r, 0);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

/* void fetch(long ctx, long[] ids, byte[] sums, int[] records) — sums: k * 24 bytes; records:
 * k*n*4 ints (decision, decisionRound, haltRound, finalX). */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_fetch(JNIEnv* env, jobject self, jlong h, jlongArray ids,
                                                                 jbyteArray sums, jintArray recs) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !check_len(env, ids, 0, 0, "ids")) return;
  const jsize k = (*env)->GetArrayLength(env, ids);
  if (!check_len(env, sums, (int64_t)k * (int64_t)sizeof(psg_instance_summary), 0, "sums") ||
      !check_len(env, recs, (int64_t)k * j->n * 4, 0, "records"))
    return;
  jlong* id = (*env)->GetLongArrayElements(env, ids, NULL);
  psg_instance_summary* s = (psg_instance_summary*)malloc(sizeof(psg_instance_summary) * (size_t)(k ? k : 1));
  jint* r = (*env)->GetIntArrayElements(env, recs, NULL);
  int rc = s ? psg_fetch_instances(j->ctx, (const uint64_t*)id, (size_t)k, s, (psg_process_record*)r) : PSG_ENOMEM;
  (*env)->ReleaseIntArrayElements(env, recs, r, 0);
  (*env)->ReleaseLongArrayElements(env, ids, id, JNI_ABORT);
  if (rc == 0) (*env)->SetByteArrayRegion(env, sums, 0, (jsize)(sizeof(*s) * (size_t)k), (const jbyte*)s);
  free(s);
  if (rc) throw_psg(env, rc, rc == PSG_ENOMEM ? "out of host memory" : psg_last_error(j->ctx));
}

/* void loadInputsF64(long ctx, long begin, long count, double[] init) — RealConsensusIO inputs */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadInputsF64(JNIEnv* env, jobject self, jlong h,
                                                                         jlong begin, jlong count, jdoubleArray init) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) || !check_len(env, init, count * j->n, 1, "init")) return;
  jdouble* p = init ? (*env)->GetDoubleArrayElements(env, init, NULL) : NULL;
  int rc = psg_load_inputs_f64(j->ctx, (uint64_t)begin, (uint64_t)count, (const double*)p);
  if (p) (*env)->ReleaseDoubleArrayElements(env, init, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

/* void copyDecisionsF64(long ctx, double[] decision, int[] round) — RealConsensusIO.decide values */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_copyDecisionsF64(JNIEnv* env, jobject self, jlong h,
                                                                            jdoubleArray dec, jintArray round) {
  (void)self;
  jctx* j = J(env, h);
  const int64_t cells = j ? last_cells(j) : 0;
  if (!j || !check_len(env, dec, cells, 1, "decision") || !check_len(env, round, cells, 1, "decisionRound")) return;
  jdouble* d = dec ? (*env)->GetDoubleArrayElements(env, dec, NULL) : NULL;
  jint* r = round ? (*env)->GetIntArrayElements(env, round, NULL) : NULL;
  int rc = psg_copy_decisions_f64(j->ctx, (double*)d, (int32_t*)r);
  if (d) (*env)->ReleaseDoubleArrayElements(env, dec, d, 0);
  if (r) (*env)->ReleaseIntArrayElements(env, round, r, 0);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

/* void loadSchedule(long ctx, long begin, long count, long[] ho, int[] crashOrNull) —
 * explicit HO sets [count][R][n][W] (psg_load_schedule) */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadSchedule(JNIEnv* env, jobject self, jlong h,
                                                                        jlong begin, jlong count, jlongArray ho,
                                                                        jintArray crash) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) ||
      !check_len(env, ho, count * j->rounds * j->n * j->words, 0, "ho") ||
      !check_len(env, crash, count * j->n, 1, "crash"))
    return;
  jlong* p = (*env)->GetLongArrayElements(env, ho, NULL);
  jint* c = crash ? (*env)->GetIntArrayElements(env, crash, NULL) : NULL;
  int rc = psg_load_schedule(j->ctx, (uint64_t)begin, (uint64_t)count, (const uint64_t*)p, (const int32_t*)c);
  if (c) (*env)->ReleaseIntArrayElements(env, crash, c, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, ho, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

/* void clearSchedule(long ctx) — back to seeded HO sets */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_clearSchedule(JNIEnv* env, jobject self, jlong h) {
  (void)self;
  jctx* j = J(env, h);
  if (!j) return;
  int rc = psg_clear_schedule(j->ctx);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

/* void materializeSchedule(long ctx, long begin, long count, long[] ho, int[] crashOrNull) — the seeded
 * HO sets as data, [count][R][n][W] and [count][n] (psg_materialize_schedule): what the in-JVM
 * harness (integration/scala/HoHarness.scala) replays through the reference's own rounds */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_materializeSchedule(JNIEnv* env, jobject self, jlong h,
                                                                               jlong begin, jlong count,
                                                                               jlongArray ho, jintArray crash) {
  (void)self;
  jctx* j = J(env, h);
  if (!j || !count_ok(env, begin, count) ||
      !check_len(env, ho, count * j->rounds * j->n * j->words, 0, "ho") ||
      !check_len(env, crash, count * j->n, 1, "crash"))
    return;
  jlong* p = (*env)->GetLongArrayElements(env, ho, NULL);
  jint* c = crash ? (*env)->GetIntArrayElements(env, crash, NULL) : NULL;
  int rc = psg_materialize_schedule(j->ctx, (uint64_t)begin, (uint64_t)count, (uint64_t*)p, (int32_t*)c);
  if (c) (*env)->ReleaseIntArrayElements(env, crash, c, 0);
  (*env)->ReleaseLongArrayElements(env, ho, p, 0);
  if (rc) throw_psg(env, rc, psg_last_error(j->ctx));
}

JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_destroy(JNIEnv* env, jobject self, jlong h) {
  (void)env;
  (void)self;
  jctx* j = (jctx*)(intptr_t)h;
  if (!j) return;
  psg_destroy(j->ctx);
  free(j);
}
