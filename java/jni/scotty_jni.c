/* scotty_jni.c -- JNI binding of the Java shim (java/main/de/tub/dima/scotty/slicing/JniApi.java), the default on
 * every JDK from 8 on.  Each native method forwards to one entry point of include/scotty_mi355x.h.
 * Tuple buffers arrive as direct ByteBuffers (GetDirectBufferAddress: the library reads the off-heap memory the
 * shim filled, no copy); a watermark's SoA result columns are copied into fresh Java arrays.
 *
 * Build (JDK 8+; no JDK exists in this repository's build container: tests/test_java_shim_cpu.py compiles this file
 * with -fsyntax-only against a type-check stub of jni.h, tests/jni_stub/jni.h, and links nothing):
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -Iinclude \
 *       java/jni/scotty_jni.c -Lscotty-window-processor_amd -lscotty_mi355x -Wl,-rpath,'$ORIGIN' \
 *       -o libscotty_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "scotty_mi355x.h"

#define OP(h) ((scotty_op*)(intptr_t)(h))

static void* addr(JNIEnv* env, jobject buf) { return buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL; }

JNIEXPORT jlong JNICALL Java_de_tub_dima_scotty_slicing_JniApi_create0(JNIEnv* env, jclass cls, jint device,
                                                                       jint value_type, jint flags, jintArray rc) {
  (void)cls;
  scotty_op* op = NULL;
  jint r = scotty_create(&op, device, value_type, (uint32_t)flags);
  (*env)->SetIntArrayRegion(env, rc, 0, 1, &r);
  return r < 0 ? 0 : (jlong)(intptr_t)op;
}

JNIEXPORT void JNICALL Java_de_tub_dima_scotty_slicing_JniApi_destroy0(JNIEnv* env, jclass cls, jlong op) {
  (void)env;
  (void)cls;
  scotty_destroy(OP(op));
}

JNIEXPORT jstring JNICALL Java_de_tub_dima_scotty_slicing_JniApi_lastError0(JNIEnv* env, jclass cls, jlong op) {
  (void)cls;
  const char* m = scotty_last_error(OP(op));
  return (*env)->NewStringUTF(env, m ? m : "");
}

JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_addWindow0(JNIEnv* env, jclass cls, jlong op, jint kind,
                                                                         jint measure, jlong a, jlong b) {
  (void)env;
  (void)cls;
  return scotty_add_window(OP(op), kind, measure, a, b);
}

JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_addAggregation0(JNIEnv* env, jclass cls, jlong op,
                                                                              jint kind) {
  (void)env;
  (void)cls;
  return scotty_add_aggregation(OP(op), kind);
}

JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_setMaxLateness0(JNIEnv* env, jclass cls, jlong op,
                                                                              jlong lateness) {
  (void)env;
  (void)cls;
  return scotty_set_max_lateness(OP(op), lateness);
}

JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_processElements0(JNIEnv* env, jclass cls, jlong op,
                                                                               jobject ts, jobject val, jlong n) {
  (void)cls;
  const void* t = addr(env, ts);
  const void* v = addr(env, val);
  if (n > 0 && (!t || !v)) return SCOTTY_ERR_ARG;  /* not a direct buffer */
  return scotty_process_elements(OP(op), (const int64_t*)t, v, (size_t)n);
}

JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_processKeyedElements0(JNIEnv* env, jclass cls, jlong op,
                                                                                    jobject key, jobject ts,
                                                                                    jobject val, jlong n) {
  (void)cls;
  const void* k = addr(env, key);
  const void* t = addr(env, ts);
  const void* v = addr(env, val);
  if (n > 0 && (!k || !t || !v)) return SCOTTY_ERR_ARG;
  return scotty_process_keyed_elements(OP(op), (const uint32_t*)k, (const int64_t*)t, v, (size_t)n);
}

static int set_longs(JNIEnv* env, jobject out, jclass oc, const char* name, const int64_t* src, jsize n) {
  jlongArray a = (*env)->NewLongArray(env, n);
  if (!a) return -1;
  if (n > 0) (*env)->SetLongArrayRegion(env, a, 0, n, (const jlong*)src);
  (*env)->SetObjectField(env, out, (*env)->GetFieldID(env, oc, name, "[J"), a);
  (*env)->DeleteLocalRef(env, a);
  return 0;
}

static int set_ints(JNIEnv* env, jobject out, jclass oc, const char* name, const int32_t* src, jsize n) {
  jintArray a = (*env)->NewIntArray(env, n);
  if (!a) return -1;
  if (n > 0) (*env)->SetIntArrayRegion(env, a, 0, n, (const jint*)src);
  (*env)->SetObjectField(env, out, (*env)->GetFieldID(env, oc, name, "[I"), a);
  (*env)->DeleteLocalRef(env, a);
  return 0;
}

/* scotty_first_indices -> long[] (null with the status in lastError0 on failure) */
JNIEXPORT jlongArray JNICALL Java_de_tub_dima_scotty_slicing_JniApi_firstIndices0(JNIEnv* env, jclass cls, jlong op) {
  (void)cls;
  const int64_t n = scotty_first_indices(OP(op), NULL, 0);
  if (n < 0) return NULL;
  jlongArray a = (*env)->NewLongArray(env, (jsize)n);
  if (!a || n == 0) return a;
  int64_t* buf = (int64_t*)malloc((size_t)n * sizeof(int64_t));
  if (!buf) return NULL;
  const int64_t m = scotty_first_indices(OP(op), buf, (size_t)n);
  if (m == n) (*env)->SetLongArrayRegion(env, a, 0, (jsize)n, (const jlong*)buf);
  free(buf);
  return m == n ? a : NULL;
}

/* scotty_process_watermark -> NativeApi.Windows {n, start, end, measure, has, values[n_aggs][n], key} */
JNIEXPORT jint JNICALL Java_de_tub_dima_scotty_slicing_JniApi_processWatermark0(JNIEnv* env, jclass cls, jlong op,
                                                                                jlong wm, jobject out) {
  (void)cls;
  scotty_windows w;
  memset(&w, 0, sizeof(w));
  const jint rc = scotty_process_watermark(OP(op), wm, &w);
  if (rc < 0) return rc;
  const jsize n = (jsize)w.n_windows;
  jclass oc = (*env)->GetObjectClass(env, out);
  (*env)->SetIntField(env, out, (*env)->GetFieldID(env, oc, "n", "I"), n);
  if (set_longs(env, out, oc, "start", w.start, n) || set_longs(env, out, oc, "end", w.end, n) ||
      set_ints(env, out, oc, "measure", w.measure, n))
    return SCOTTY_ERR_NOMEM;
  jbyteArray has = (*env)->NewByteArray(env, n);
  if (!has) return SCOTTY_ERR_NOMEM;
  if (n > 0) (*env)->SetByteArrayRegion(env, has, 0, n, (const jbyte*)w.has_value);
  (*env)->SetObjectField(env, out, (*env)->GetFieldID(env, oc, "has", "[B"), has);
  (*env)->DeleteLocalRef(env, has);
  jclass lac = (*env)->FindClass(env, "[J");
  jobjectArray vals = (*env)->NewObjectArray(env, w.n_aggs, lac, NULL);
  if (!vals) return SCOTTY_ERR_NOMEM;
  for (jsize k = 0; k < w.n_aggs; k++) {
    jlongArray a = (*env)->NewLongArray(env, n);
    if (!a) return SCOTTY_ERR_NOMEM;
    if (n > 0) (*env)->SetLongArrayRegion(env, a, 0, n, (const jlong*)w.values[k]);
    (*env)->SetObjectArrayElement(env, vals, k, a);
    (*env)->DeleteLocalRef(env, a);
  }
  (*env)->SetObjectField(env, out, (*env)->GetFieldID(env, oc, "values", "[[J"), vals);
  (*env)->DeleteLocalRef(env, vals);
  if (w.key) {
    if (set_ints(env, out, oc, "key", (const int32_t*)w.key, n)) return SCOTTY_ERR_NOMEM;
  } else {
    (*env)->SetObjectField(env, out, (*env)->GetFieldID(env, oc, "key", "[I"), NULL);
  }
  return rc;
}
