/*
 * psg_jni.c — JNI binding of include/psg.h for the Scala `psync.gpu.GpuRound`
 * plugin (integration/scala/GpuRound.scala).
 *
 * Not built in this container (no JDK / jni.h). On a machine with a JDK:
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" \
 *       -I<repo>/include psg_jni.c -L<repo>/round_amd -lpsg -Wl,-rpath,<repo>/round_amd \
 *       -o libpsg_jni.so
 * and load it with System.loadLibrary("psg_jni").
 *
 * Each native method maps 1:1 onto a C-ABI entry point; errors become
 * java.lang.IllegalStateException / IllegalArgumentException carrying
 * psg_last_error(), mirroring the reference's Logger.logAndThrow
 * (psync/runtime/InstanceHandler.scala:346, 351).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "psg.h"

static void throw_psg(JNIEnv* env, int rc, const char* msg) {
  const char* cls = rc == PSG_EINVAL || rc == PSG_ERANGE ? "java/lang/IllegalArgumentException"
                                                          : "java/lang/IllegalStateException";
  jclass ex = (*env)->FindClass(env, cls);
  char buf[512];
  snprintf(buf, sizeof buf, "psg error %d: %s", rc, msg ? msg : "");
  if (ex) (*env)->ThrowNew(env, ex, buf);
}

/* long create(int alg, int n, int rounds, long seed, int valueRange, int param, int param2, double realParam,
 *             int tiebreak, int device, int variant, long batchCapacity,
 *             int dropLog2, int goodP32, int goodMin, int crashFmax, int hoMin, boolean selfBit) */
JNIEXPORT jlong JNICALL Java_psync_gpu_GpuRoundNative_00024_create(
    JNIEnv* env, jobject self, jint alg, jint n, jint rounds, jlong seed, jint valueRange, jint param, jint param2,
    jdouble realParam, jint tiebreak, jint device, jint variant, jlong batchCapacity, jint dropLog2, jint goodP32,
    jint goodMin, jint crashFmax, jint hoMin, jboolean selfBit) {
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
  psg_ctx* ctx = NULL;
  int rc = psg_create(&ctx, &c);
  if (rc) {
    throw_psg(env, rc, psg_create_error());
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

/* void loadInputs(long ctx, long begin, long count, int[] init) — init may be null (seeded) */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadInputs(JNIEnv* env, jobject self, jlong h,
                                                                      jlong begin, jlong count, jintArray init) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jint* p = init ? (*env)->GetIntArrayElements(env, init, NULL) : NULL;
  int rc = psg_load_inputs(ctx, (uint64_t)begin, (uint64_t)count, (const int32_t*)p);
  if (p) (*env)->ReleaseIntArrayElements(env, init, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* long[] runBatch(long ctx, long begin, long count, byte[] perInstanceOrNull)
 * returns the psg_summary as a flat long[] (struct order); perInstance receives
 * count * sizeof(psg_instance_summary) bytes when non-null. */
JNIEXPORT jlongArray JNICALL Java_psync_gpu_GpuRoundNative_00024_runBatch(JNIEnv* env, jobject self, jlong h,
                                                                          jlong begin, jlong count,
                                                                          jbyteArray perInst) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  psg_summary s;
  psg_instance_summary* pi = NULL;
  if (perInst) {
    pi = (psg_instance_summary*)malloc(sizeof(psg_instance_summary) * (size_t)count);
    if (!pi) {
      throw_psg(env, PSG_ENOMEM, "out of host memory");
      return NULL;
    }
  }
  int rc = psg_run_batch(ctx, (uint64_t)begin, (uint64_t)count, &s, pi);
  if (rc) {
    free(pi);
    throw_psg(env, rc, psg_last_error(ctx));
    return NULL;
  }
  if (perInst) {
    (*env)->SetByteArrayRegion(env, perInst, 0, (jsize)(sizeof(psg_instance_summary) * (size_t)count),
                               (const jbyte*)pi);
    free(pi);
  }
  const jsize len = (jsize)(sizeof(psg_summary) / sizeof(int64_t));
  jlongArray out = (*env)->NewLongArray(env, len);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, len, (const jlong*)&s);
  return out;
}

/* void copyDecisions(long ctx, int[] decision, int[] decisionRound) — the batched
 * ConsensusIO.decide results of the last batch, [count][n] each. */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_copyDecisions(JNIEnv* env, jobject self, jlong h,
                                                                         jintArray dec, jintArray drnd) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jint* d = (*env)->GetIntArrayElements(env, dec, NULL);
  jint* r = (*env)->GetIntArrayElements(env, drnd, NULL);
  int rc = psg_copy_decisions(ctx, (int32_t*)d, (int32_t*)r);
  (*env)->ReleaseIntArrayElements(env, dec, d, 0);
  (*env)->ReleaseIntArrayElements(env, drnd, r, 0);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void fetch(long ctx, long[] ids, byte[] sums, int[] records) — records: k*n*4 ints
 * (decision, decisionRound, haltRound, finalX). */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_fetch(JNIEnv* env, jobject self, jlong h, jlongArray ids,
                                                                 jbyteArray sums, jintArray recs) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  const jsize k = (*env)->GetArrayLength(env, ids);
  jlong* id = (*env)->GetLongArrayElements(env, ids, NULL);
  psg_instance_summary* s = (psg_instance_summary*)malloc(sizeof(psg_instance_summary) * (size_t)(k ? k : 1));
  jint* r = (*env)->GetIntArrayElements(env, recs, NULL);
  int rc = s ? psg_fetch_instances(ctx, (const uint64_t*)id, (size_t)k, s, (psg_process_record*)r) : PSG_ENOMEM;
  (*env)->ReleaseIntArrayElements(env, recs, r, 0);
  (*env)->ReleaseLongArrayElements(env, ids, id, JNI_ABORT);
  if (rc == 0) (*env)->SetByteArrayRegion(env, sums, 0, (jsize)(sizeof(*s) * (size_t)k), (const jbyte*)s);
  free(s);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void loadInputsF64(long ctx, long begin, long count, double[] init) — RealConsensusIO inputs */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadInputsF64(JNIEnv* env, jobject self, jlong h,
                                                                         jlong begin, jlong count, jdoubleArray init) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jdouble* p = init ? (*env)->GetDoubleArrayElements(env, init, NULL) : NULL;
  int rc = psg_load_inputs_f64(ctx, (uint64_t)begin, (uint64_t)count, (const double*)p);
  if (p) (*env)->ReleaseDoubleArrayElements(env, init, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void copyDecisionsF64(long ctx, double[] decision, int[] round) — RealConsensusIO.decide values */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_copyDecisionsF64(JNIEnv* env, jobject self, jlong h,
                                                                            jdoubleArray dec, jintArray round) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jdouble* d = (*env)->GetDoubleArrayElements(env, dec, NULL);
  jint* r = (*env)->GetIntArrayElements(env, round, NULL);
  int rc = psg_copy_decisions_f64(ctx, (double*)d, (int32_t*)r);
  (*env)->ReleaseDoubleArrayElements(env, dec, d, 0);
  (*env)->ReleaseIntArrayElements(env, round, r, 0);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void loadSchedule(long ctx, long begin, long count, long[] ho, int[] crashOrNull) —
 * explicit HO sets [count][R][n][W] (psg_load_schedule) */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_loadSchedule(JNIEnv* env, jobject self, jlong h,
                                                                        jlong begin, jlong count, jlongArray ho,
                                                                        jintArray crash) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jlong* p = (*env)->GetLongArrayElements(env, ho, NULL);
  jint* c = crash ? (*env)->GetIntArrayElements(env, crash, NULL) : NULL;
  int rc = psg_load_schedule(ctx, (uint64_t)begin, (uint64_t)count, (const uint64_t*)p, (const int32_t*)c);
  if (c) (*env)->ReleaseIntArrayElements(env, crash, c, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, ho, p, JNI_ABORT);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void clearSchedule(long ctx) — back to seeded HO sets */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_clearSchedule(JNIEnv* env, jobject self, jlong h) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  int rc = psg_clear_schedule(ctx);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

/* void materializeSchedule(long ctx, long begin, long count, long[] ho, int[] crash) — the seeded
 * HO sets as data, [count][R][n][W] and [count][n] (psg_materialize_schedule): what the in-JVM
 * harness (integration/scala/HoHarness.scala) replays through the reference's own rounds */
JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_materializeSchedule(JNIEnv* env, jobject self, jlong h,
                                                                               jlong begin, jlong count,
                                                                               jlongArray ho, jintArray crash) {
  (void)self;
  psg_ctx* ctx = (psg_ctx*)(intptr_t)h;
  jlong* p = (*env)->GetLongArrayElements(env, ho, NULL);
  jint* c = crash ? (*env)->GetIntArrayElements(env, crash, NULL) : NULL;
  int rc = psg_materialize_schedule(ctx, (uint64_t)begin, (uint64_t)count, (uint64_t*)p, (int32_t*)c);
  if (c) (*env)->ReleaseIntArrayElements(env, crash, c, 0);
  (*env)->ReleaseLongArrayElements(env, ho, p, 0);
  if (rc) throw_psg(env, rc, psg_last_error(ctx));
}

JNIEXPORT void JNICALL Java_psync_gpu_GpuRoundNative_00024_destroy(JNIEnv* env, jobject self, jlong h) {
  (void)env;
  (void)self;
  psg_destroy((psg_ctx*)(intptr_t)h);
}
