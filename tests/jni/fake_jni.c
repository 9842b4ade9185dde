/*
 * fake_jni.c — test infrastructure: a JNIEnv implemented in C over plain heap objects,
 * so the JNI shim integration/jni/psg_jni.c can be EXECUTED without a JVM (the image
 * has none). Built together with the shim against integration/jni/jni_min/jni.h into
 * tests/jni/libpsg_jni_test.so (tests/jni/Makefile) and driven through ctypes by
 * tests/test_jni_shim.py: Java arrays and strings are FjObj records, ThrowNew records
 * the pending exception, and every region copy is bounds-checked (an out-of-bounds
 * access sets a flag instead of touching memory). Not a JVM: it exercises the shim's
 * marshalling, argument checks and C-ABI calls, not the JVM's own conventions.
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { FJ_INT = 1, FJ_LONG = 2, FJ_BYTE = 3, FJ_DOUBLE = 4, FJ_STRING = 5, FJ_CLASS = 6 };
typedef struct FjObj {
  int kind;
  jsize len;
  void* data;
} FjObj;

static char g_cls[256], g_msg[1024];
static int g_pending = 0, g_oob = 0;

static size_t esize(int kind) {
  switch (kind) {
    case FJ_INT: return 4;
    case FJ_LONG: return 8;
    case FJ_DOUBLE: return 8;
    default: return 1;
  }
}
static FjObj* mk(int kind, jsize len) {
  FjObj* o = (FjObj*)calloc(1, sizeof(FjObj));
  o->kind = kind;
  o->len = len;
  o->data = calloc((size_t)(len > 0 ? len : 1) + (kind == FJ_STRING ? 1 : 0), esize(kind));
  return o;
}
static int region_ok(jarray a, jsize start, jsize len) {
  const FjObj* o = (const FjObj*)a;
  if (!o || start < 0 || len < 0 || start + len > o->len) {
    g_oob = 1;
    return 0;
  }
  return 1;
}

static jclass FindClass(JNIEnv* env, const char* name) {
  (void)env;
  FjObj* o = mk(FJ_CLASS, (jsize)strlen(name));
  memcpy(o->data, name, strlen(name));
  return (jclass)o;
}
static jint ThrowNew(JNIEnv* env, jclass c, const char* msg) {
  (void)env;
  snprintf(g_cls, sizeof g_cls, "%s", (const char*)((FjObj*)c)->data);
  snprintf(g_msg, sizeof g_msg, "%s", msg ? msg : "");
  g_pending = 1;
  return 0;
}
static jsize GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  return ((FjObj*)a)->len;
}
static jlongArray NewLongArray(JNIEnv* env, jsize len) {
  (void)env;
  return (jlongArray)mk(FJ_LONG, len);
}
static jintArray NewIntArray(JNIEnv* env, jsize len) {
  (void)env;
  return (jintArray)mk(FJ_INT, len);
}
static jint* GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* c) {
  (void)env;
  if (c) *c = 0;
  return (jint*)((FjObj*)a)->data;
}
static jlong* GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* c) {
  (void)env;
  if (c) *c = 0;
  return (jlong*)((FjObj*)a)->data;
}
static jdouble* GetDoubleArrayElements(JNIEnv* env, jdoubleArray a, jboolean* c) {
  (void)env;
  if (c) *c = 0;
  return (jdouble*)((FjObj*)a)->data;
}
static void ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* e, jint m) { (void)env; (void)a; (void)e; (void)m; }
static void ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* e, jint m) { (void)env; (void)a; (void)e; (void)m; }
static void ReleaseDoubleArrayElements(JNIEnv* env, jdoubleArray a, jdouble* e, jint m) {
  (void)env; (void)a; (void)e; (void)m;
}
static void GetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, jint* buf) {
  (void)env;
  if (region_ok(a, s, n)) memcpy(buf, (jint*)((FjObj*)a)->data + s, sizeof(jint) * (size_t)n);
}
static void SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize s, jsize n, const jbyte* buf) {
  (void)env;
  if (region_ok(a, s, n)) memcpy((jbyte*)((FjObj*)a)->data + s, buf, (size_t)n);
}
static void SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize s, jsize n, const jlong* buf) {
  (void)env;
  if (region_ok(a, s, n)) memcpy((jlong*)((FjObj*)a)->data + s, buf, sizeof(jlong) * (size_t)n);
}
static void SetIntArrayRegion(JNIEnv* env, jintArray a, jsize s, jsize n, const jint* buf) {
  (void)env;
  if (region_ok(a, s, n)) memcpy((jint*)((FjObj*)a)->data + s, buf, sizeof(jint) * (size_t)n);
}
static jstring NewStringUTF(JNIEnv* env, const char* utf) {
  (void)env;
  FjObj* o = mk(FJ_STRING, (jsize)strlen(utf));
  memcpy(o->data, utf, strlen(utf));
  return (jstring)o;
}
static const char* GetStringUTFChars(JNIEnv* env, jstring s, jboolean* c) {
  (void)env;
  if (c) *c = 0;
  return (const char*)((FjObj*)s)->data;
}
static void ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* ch) { (void)env; (void)s; (void)ch; }

static const struct JNINativeInterface_ g_table = {
    .FindClass = FindClass, .ThrowNew = ThrowNew, .GetArrayLength = GetArrayLength, .NewLongArray = NewLongArray,
    .GetIntArrayElements = GetIntArrayElements, .GetLongArrayElements = GetLongArrayElements,
    .GetDoubleArrayElements = GetDoubleArrayElements, .ReleaseIntArrayElements = ReleaseIntArrayElements,
    .ReleaseLongArrayElements = ReleaseLongArrayElements, .ReleaseDoubleArrayElements = ReleaseDoubleArrayElements,
    .GetIntArrayRegion = GetIntArrayRegion, .SetByteArrayRegion = SetByteArrayRegion,
    .SetLongArrayRegion = SetLongArrayRegion, .NewIntArray = NewIntArray, .SetIntArrayRegion = SetIntArrayRegion,
    .NewStringUTF = NewStringUTF, .GetStringUTFChars = GetStringUTFChars,
    .ReleaseStringUTFChars = ReleaseStringUTFChars};
static JNIEnv g_env = &g_table;

/* ---- ctypes surface ---- */
JNIEnv* fj_env(void) { return &g_env; }
void* fj_new(int kind, int len) { return mk(kind, len); }
void* fj_string(const char* s) { return NewStringUTF(&g_env, s); }
void* fj_data(void* o) { return ((FjObj*)o)->data; }
int fj_len(void* o) { return ((FjObj*)o)->len; }
void fj_free(void* o) {
  if (!o) return;
  free(((FjObj*)o)->data);
  free(o);
}
/* 1 and the exception's class / message if one is pending (then cleared), else 0 */
int fj_take_exception(char* cls, size_t cl, char* msg, size_t ml) {
  if (!g_pending) return 0;
  snprintf(cls, cl, "%s", g_cls);
  snprintf(msg, ml, "%s", g_msg);
  g_pending = 0;
  return 1;
}
int fj_take_oob(void) {
  const int r = g_oob;
  g_oob = 0;
  return r;
}
/* a context handle of the shim's layout with no psg context behind it (argument-check tests) */
typedef struct { void* ctx; long long n, rounds, words; } fj_jctx;
void* fj_fake_ctx(int n, int rounds) {
  fj_jctx* j = (fj_jctx*)calloc(1, sizeof(fj_jctx));
  j->n = n;
  j->rounds = rounds;
  j->words = (n + 63) / 64;
  return j;
}
