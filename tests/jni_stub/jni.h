/* jni.h -- TYPE-CHECK STUB for tests/test_java_shim_cpu.py, not a JDK header.
 *
 * No JDK exists in the build container, so the JNI binding java/jni/scotty_jni.c is compiled here with
 * gcc -fsyntax-only against this stub: the JNI types and exactly the JNIEnv functions that file calls, with the
 * signatures of the JNI specification (Java Native Interface Specification, "JNI Functions").  The member order is
 * not the real function table's, so nothing compiled against this file may be linked or run: a real build uses
 * $JAVA_HOME/include. */
#ifndef SCOTTY_TEST_JNI_STUB_H
#define SCOTTY_TEST_JNI_STUB_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jbyteArray;
typedef jarray jobjectArray;
struct _jfieldID;
typedef struct _jfieldID* jfieldID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);
  void(JNICALL* DeleteLocalRef)(JNIEnv* env, jobject obj);
  jclass(JNICALL* GetObjectClass)(JNIEnv* env, jobject obj);
  jfieldID(JNICALL* GetFieldID)(JNIEnv* env, jclass clazz, const char* name, const char* sig);
  void(JNICALL* SetObjectField)(JNIEnv* env, jobject obj, jfieldID fieldID, jobject val);
  void(JNICALL* SetIntField)(JNIEnv* env, jobject obj, jfieldID fieldID, jint val);
  jstring(JNICALL* NewStringUTF)(JNIEnv* env, const char* utf);
  jobjectArray(JNICALL* NewObjectArray)(JNIEnv* env, jsize len, jclass clazz, jobject init);
  void(JNICALL* SetObjectArrayElement)(JNIEnv* env, jobjectArray array, jsize index, jobject val);
  jbyteArray(JNICALL* NewByteArray)(JNIEnv* env, jsize len);
  jintArray(JNICALL* NewIntArray)(JNIEnv* env, jsize len);
  jlongArray(JNICALL* NewLongArray)(JNIEnv* env, jsize len);
  void(JNICALL* SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
  void(JNICALL* SetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf);
  void(JNICALL* SetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, const jlong* buf);
  void*(JNICALL* GetDirectBufferAddress)(JNIEnv* env, jobject buf);
};

#endif
