/*
 * jni.h -- TEST-ONLY minimal JNI header (tests/jni), NOT a JDK header.
 *
 * There is no JDK in the build image, so integration/jni/cfk_als_jni.c is compiled here against this header to be
 * executed by a mock JVM (mock_jvm.c) from the tests. It declares only the JNI types and the JNINativeInterface_
 * members the shim uses, with the JNI specification's signatures (so the same shim source compiles unchanged against
 * a real $JAVA_HOME/include/jni.h). Member order is NOT the real function table's: the shim calls members by name
 * (`(*env)->GetArrayLength(env, a)`), which is all the C source depends on.
 */
#ifndef CFK_TEST_JNI_H
#define CFK_TEST_JNI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_COMMIT 1
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
    jclass(JNICALL* FindClass)(JNIEnv* env, const char* name);
    jint(JNICALL* ThrowNew)(JNIEnv* env, jclass clazz, const char* msg);
    jboolean(JNICALL* ExceptionCheck)(JNIEnv* env);
    jsize(JNICALL* GetArrayLength)(JNIEnv* env, jarray array);
    void*(JNICALL* GetPrimitiveArrayCritical)(JNIEnv* env, jarray array, jboolean* isCopy);
    void(JNICALL* ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray array, void* carray, jint mode);
    jbyteArray(JNICALL* NewByteArray)(JNIEnv* env, jsize len);
    void(JNICALL* GetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf);
    void(JNICALL* SetByteArrayRegion)(JNIEnv* env, jbyteArray array, jsize start, jsize len, const jbyte* buf);
    void(JNICALL* GetShortArrayRegion)(JNIEnv* env, jshortArray array, jsize start, jsize len, jshort* buf);
    void(JNICALL* GetIntArrayRegion)(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf);
    void(JNICALL* GetLongArrayRegion)(JNIEnv* env, jlongArray array, jsize start, jsize len, jlong* buf);
    void(JNICALL* GetFloatArrayRegion)(JNIEnv* env, jfloatArray array, jsize start, jsize len, jfloat* buf);
    void(JNICALL* SetFloatArrayRegion)(JNIEnv* env, jfloatArray array, jsize start, jsize len, const jfloat* buf);
    void(JNICALL* GetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, jdouble* buf);
    void(JNICALL* SetDoubleArrayRegion)(JNIEnv* env, jdoubleArray array, jsize start, jsize len, const jdouble* buf);
    jfloat*(JNICALL* GetFloatArrayElements)(JNIEnv* env, jfloatArray array, jboolean* isCopy);
    void(JNICALL* ReleaseFloatArrayElements)(JNIEnv* env, jfloatArray array, jfloat* elems, jint mode);
    const char*(JNICALL* GetStringUTFChars)(JNIEnv* env, jstring str, jboolean* isCopy);
    void(JNICALL* ReleaseStringUTFChars)(JNIEnv* env, jstring str, const char* chars);
};

#ifdef __cplusplus
}
#endif
#endif /* CFK_TEST_JNI_H */
