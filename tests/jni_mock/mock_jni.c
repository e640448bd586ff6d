/* mock_jni.c -- a FUNCTIONAL mock of the JNIEnv the Java shim's JNI binding (java/jni/scotty_jni.c) calls, so the
 * binding's marshalling runs end to end without a JDK (none exists in the build container or on the GPU box).
 *
 * Test infrastructure only.  Built by tests/jni_mock/Makefile into libjni_mock.so together with java/jni/scotty_jni.c,
 * both compiled against the type-check stub tests/jni_stub/jni.h (the same function table on both sides), linked
 * against the product library.  tests/test_jni_binding.py drives the JNI entry points exactly as JniApi.java and
 * SlicingWindowOperator.java / KeyedEngine.java call them (direct ByteBuffers filled off-heap, one
 * NativeApi.Windows object per watermark) and checks the rows against the CPU oracle.
 *
 * Object model: every jobject is a struct mobj.  Arrays own their elements; a direct ByteBuffer wraps the caller's
 * memory (GetDirectBufferAddress returns it, NULL for a heap buffer as in the JVM); a Windows object holds the seven
 * fields of NativeApi.Windows, and GetFieldID resolves only those (name AND signature, as the JVM does -- a wrong
 * signature yields NULL and a pending NoSuchFieldError).  Local references are counted: every New*Array /
 * NewStringUTF / GetObjectClass / FindClass result is one, DeleteLocalRef releases one, so a test can see how many
 * the binding leaves for the JVM to reclaim when the native method returns.  Out-of-range array regions raise a
 * pending ArrayIndexOutOfBoundsException (recorded, not thrown: the harness asserts none is pending). */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { M_CLASS = 1, M_STRING, M_DBUF, M_HEAPBUF, M_LONGS, M_INTS, M_BYTES, M_OBJS, M_WINDOWS };

struct _jobject {
  int kind;
  jsize n;                 /* array length / string length */
  void* data;              /* array elements, string bytes, direct buffer address */
  struct _jobject* fields[7];  /* M_WINDOWS: start end measure has values key (by FIELD_*); n in wn */
  jint wn;
  const char* cname;       /* M_CLASS: class name */
  struct _jobject* next;   /* every object, for mock_reset */
};

struct _jfieldID {
  const char* name;
  const char* sig;
  int slot;  /* -1: the int field n */
};

/* NativeApi.Windows (java/main/de/tub/dima/scotty/slicing/NativeApi.java) */
static const struct _jfieldID FIELDS[] = {
    {"n", "I", -1}, {"start", "[J", 0}, {"end", "[J", 1}, {"measure", "[I", 2},
    {"has", "[B", 3}, {"values", "[[J", 4}, {"key", "[I", 5},
};

static struct _jobject* g_all = NULL;
static int g_local_refs = 0;
static int g_exceptions = 0;
static char g_last_exception[256];

static struct _jobject* mk(int kind) {
  struct _jobject* o = (struct _jobject*)calloc(1, sizeof(struct _jobject));
  o->kind = kind;
  o->next = g_all;
  g_all = o;
  return o;
}

static void raise_exc(const char* what) {
  g_exceptions++;
  strncpy(g_last_exception, what, sizeof(g_last_exception) - 1);
}

static struct _jobject WINDOWS_CLASS = {M_CLASS, 0, NULL, {NULL}, 0, "de/tub/dima/scotty/slicing/NativeApi$Windows",
                                        NULL};

static jclass JNICALL m_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  struct _jobject* c = mk(M_CLASS);
  c->cname = name;
  g_local_refs++;
  return c;
}
static void JNICALL m_DeleteLocalRef(JNIEnv* env, jobject obj) {
  (void)env;
  if (obj) g_local_refs--;
}
static jclass JNICALL m_GetObjectClass(JNIEnv* env, jobject obj) {
  (void)env;
  g_local_refs++;
  return obj && obj->kind == M_WINDOWS ? &WINDOWS_CLASS : mk(M_CLASS);
}
static jfieldID JNICALL m_GetFieldID(JNIEnv* env, jclass clazz, const char* name, const char* sig) {
  (void)env;
  if (clazz != &WINDOWS_CLASS) {
    raise_exc("NoSuchFieldError: class is not NativeApi.Windows");
    return NULL;
  }
  for (size_t i = 0; i < sizeof(FIELDS) / sizeof(FIELDS[0]); i++)
    if (strcmp(FIELDS[i].name, name) == 0 && strcmp(FIELDS[i].sig, sig) == 0) return (jfieldID)&FIELDS[i];
  raise_exc("NoSuchFieldError: field name or signature");
  return NULL;
}
static void JNICALL m_SetObjectField(JNIEnv* env, jobject obj, jfieldID f, jobject val) {
  (void)env;
  if (!obj || obj->kind != M_WINDOWS || !f || f->slot < 0) {
    raise_exc("SetObjectField: bad object or field");
    return;
  }
  static const int want[6] = {M_LONGS, M_LONGS, M_INTS, M_BYTES, M_OBJS, M_INTS};
  if (val && val->kind != want[f->slot]) {
    raise_exc("SetObjectField: value of the wrong array type");
    return;
  }
  obj->fields[f->slot] = val;
}
static void JNICALL m_SetIntField(JNIEnv* env, jobject obj, jfieldID f, jint val) {
  (void)env;
  if (!obj || obj->kind != M_WINDOWS || !f || f->slot != -1) {
    raise_exc("SetIntField: bad object or field");
    return;
  }
  obj->wn = val;
}
static jstring JNICALL m_NewStringUTF(JNIEnv* env, const char* utf) {
  (void)env;
  struct _jobject* s = mk(M_STRING);
  s->n = (jsize)strlen(utf);
  s->data = malloc((size_t)s->n + 1);
  memcpy(s->data, utf, (size_t)s->n + 1);
  g_local_refs++;
  return s;
}
static jobject new_array(int kind, jsize len, size_t elem) {
  if (len < 0) {
    raise_exc("NegativeArraySizeException");
    return NULL;
  }
  struct _jobject* a = mk(kind);
  a->n = len;
  a->data = calloc((size_t)(len > 0 ? len : 1), elem);
  g_local_refs++;
  return a;
}
static jobjectArray JNICALL m_NewObjectArray(JNIEnv* env, jsize len, jclass clazz, jobject init) {
  (void)env;
  if (!clazz || clazz->kind != M_CLASS || strcmp(clazz->cname, "[J") != 0) raise_exc("NewObjectArray: element class");
  jobject a = new_array(M_OBJS, len, sizeof(jobject));
  for (jsize i = 0; a && i < len; i++) ((jobject*)a->data)[i] = init;
  return a;
}
static void JNICALL m_SetObjectArrayElement(JNIEnv* env, jobjectArray array, jsize index, jobject val) {
  (void)env;
  if (!array || array->kind != M_OBJS || index < 0 || index >= array->n) {
    raise_exc("ArrayIndexOutOfBoundsException: SetObjectArrayElement");
    return;
  }
  ((jobject*)array->data)[index] = val;
}
static jbyteArray JNICALL m_NewByteArray(JNIEnv* env, jsize len) {
  (void)env;
  return new_array(M_BYTES, len, 1);
}
static jintArray JNICALL m_NewIntArray(JNIEnv* env, jsize len) {
  (void)env;
  return new_array(M_INTS, len, 4);
}
static jlongArray JNICALL m_NewLongArray(JNIEnv* env, jsize len) {
  (void)env;
  return new_array(M_LONGS, len, 8);
}
static void set_region(jobject a, int kind, jsize start, jsize len, const void* buf, size_t elem) {
  if (!a || a->kind != kind) {
    raise_exc("Set<Type>ArrayRegion: wrong array type");
    return;
  }
  if (start < 0 || len < 0 || start > a->n - len) {
    raise_exc("ArrayIndexOutOfBoundsException: Set<Type>ArrayRegion");
    return;
  }
  if (len > 0) memcpy((char*)a->data + (size_t)start * elem, buf, (size_t)len * elem);
}
static void JNICALL m_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf) {
  (void)env;
  set_region(a, M_BYTES, start, len, buf, 1);
}
static void JNICALL m_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, const jint* buf) {
  (void)env;
  set_region(a, M_INTS, start, len, buf, 4);
}
static void JNICALL m_SetLongArrayRegion(JNIEnv* env, jlongArray a, jsize start, jsize len, const jlong* buf) {
  (void)env;
  set_region(a, M_LONGS, start, len, buf, 8);
}
static void* JNICALL m_GetDirectBufferAddress(JNIEnv* env, jobject buf) {
  (void)env;
  return buf && buf->kind == M_DBUF ? buf->data : NULL;  /* a heap ByteBuffer has no address */
}

static const struct JNINativeInterface_ TABLE = {
    m_FindClass,       m_DeleteLocalRef,       m_GetObjectClass, m_GetFieldID,        m_SetObjectField,
    m_SetIntField,     m_NewStringUTF,         m_NewObjectArray, m_SetObjectArrayElement, m_NewByteArray,
    m_NewIntArray,     m_NewLongArray,         m_SetByteArrayRegion, m_SetIntArrayRegion, m_SetLongArrayRegion,
    m_GetDirectBufferAddress,
};
static JNIEnv ENV = &TABLE;

/* ---- harness API (ctypes) */
JNIEXPORT JNIEnv* mock_env(void) { return &ENV; }
JNIEXPORT jobject mock_direct_buffer(void* addr, jlong capacity) {
  struct _jobject* b = mk(M_DBUF);
  b->data = addr;
  b->n = (jsize)(capacity > 0x7fffffff ? 0x7fffffff : capacity);
  return b;
}
JNIEXPORT jobject mock_heap_buffer(void) { return mk(M_HEAPBUF); }
JNIEXPORT jobject mock_int_array(jsize n) {
  jobject a = new_array(M_INTS, n, 4);
  g_local_refs--;  /* the harness's own (a Java-side `new int[1]`), not a reference the binding made */
  return a;
}
JNIEXPORT jobject mock_windows(void) { return mk(M_WINDOWS); }
JNIEXPORT jint mock_windows_n(jobject w) { return w->wn; }
/* field slot of NativeApi.Windows: 0 start, 1 end, 2 measure, 3 has, 4 values, 5 key */
JNIEXPORT jobject mock_windows_field(jobject w, int slot) { return w->fields[slot]; }
JNIEXPORT int mock_kind(jobject o) { return o ? o->kind : 0; }
JNIEXPORT jsize mock_length(jobject a) { return a->n; }
JNIEXPORT void* mock_data(jobject a) { return a->data; }
JNIEXPORT jobject mock_element(jobject a, jsize i) { return ((jobject*)a->data)[i]; }
JNIEXPORT int mock_local_refs(void) { return g_local_refs; }
JNIEXPORT int mock_exceptions(void) { return g_exceptions; }
JNIEXPORT const char* mock_last_exception(void) { return g_last_exception; }
/* frees every object; resets the reference and exception counters */
JNIEXPORT void mock_reset(void) {
  while (g_all) {
    struct _jobject* o = g_all;
    g_all = o->next;
    if (o->kind != M_DBUF && o->kind != M_CLASS) free(o->data);
    free(o);
  }
  g_local_refs = 0;
  g_exceptions = 0;
  g_last_exception[0] = 0;
}
