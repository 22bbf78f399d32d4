/*
 * mock_jvm.c -- TEST INFRASTRUCTURE: a mock JVM for executing integration/jni/cfk_als_jni.c without a JDK.
 *
 * Implements the JNINativeInterface_ members of the test-only jni.h over plain C objects that the tests create
 * through the mock_* functions below (ctypes): primitive arrays, strings, classes, and one JNIEnv per host thread
 * (JNI environments are per thread). It behaves like a copying JVM, so the shim's contract is checked, not assumed:
 *   - Get<Type>ArrayElements / GetPrimitiveArrayCritical return COPIES; the release mode decides whether they are
 *     written back (0, JNI_COMMIT) or dropped (JNI_ABORT): a wrong mode on an output array loses the data;
 *   - <Type>ArrayRegion calls are bounds- and type-checked and throw ArrayIndexOutOfBoundsException /
 *     ArrayStoreException like the JVM;
 *   - ThrowNew leaves a pending exception on the env (the test reads and clears it after each native call);
 *   - a JNI call made while an exception is pending (other than ExceptionCheck and releases) or inside a critical
 *     region, and a type mismatch, count as contract violations (mock_env_stats).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { T_BYTE = 1, T_SHORT = 2, T_INT = 3, T_LONG = 4, T_FLOAT = 5, T_DOUBLE = 6, T_STRING = 7, T_CLASS = 8 };
static const size_t ELEM[] = {0, 1, 2, 4, 8, 4, 8, 1, 1};

typedef struct {
    int type;
    jsize len;
    void* data;   /* array elements, string bytes (NUL-terminated) or class name */
} MockObj;

typedef struct {
    const struct JNINativeInterface_* fn;   /* must stay first: JNIEnv* points here */
    int pending;
    char exc_class[256];
    char exc_msg[2048];
    int in_critical;
    long n_calls, n_critical, n_copies, violations;
} MockEnv;

#define ME(env) ((MockEnv*)(env))
#define OBJ(o) ((MockObj*)(o))

static void violation(JNIEnv* env) { ME(env)->violations++; }
/* every JNI call: counts it; a call with an exception pending or inside a critical region is a violation */
static void enter(JNIEnv* env, int allowed_when_pending) {
    MockEnv* e = ME(env);
    e->n_calls++;
    if (e->pending && !allowed_when_pending) e->violations++;
    if (e->in_critical) e->violations++;
}
static void throw_(JNIEnv* env, const char* cls, const char* msg) {
    MockEnv* e = ME(env);
    if (e->pending) return;   /* the first exception wins, as in the JVM */
    e->pending = 1;
    snprintf(e->exc_class, sizeof e->exc_class, "%s", cls);
    snprintf(e->exc_msg, sizeof e->exc_msg, "%s", msg ? msg : "");
}

/* ---- class registry (FindClass returns one object per name) ---- */
static pthread_mutex_t g_cls_mu = PTHREAD_MUTEX_INITIALIZER;
static MockObj* g_classes[64];
static int g_n_classes = 0;

static jclass JNICALL m_FindClass(JNIEnv* env, const char* name) {
    enter(env, 0);
    pthread_mutex_lock(&g_cls_mu);
    MockObj* found = NULL;
    for (int i = 0; i < g_n_classes; ++i)
        if (!strcmp((const char*)g_classes[i]->data, name)) found = g_classes[i];
    if (!found && g_n_classes < 64) {
        found = calloc(1, sizeof *found);
        found->type = T_CLASS;
        found->data = strdup(name);
        found->len = (jsize)strlen(name);
        g_classes[g_n_classes++] = found;
    }
    pthread_mutex_unlock(&g_cls_mu);
    return (jclass)found;
}
static jint JNICALL m_ThrowNew(JNIEnv* env, jclass clazz, const char* msg) {
    enter(env, 0);
    if (!clazz || OBJ(clazz)->type != T_CLASS) {
        violation(env);
        return -1;
    }
    throw_(env, (const char*)OBJ(clazz)->data, msg);
    return JNI_OK;
}
static jboolean JNICALL m_ExceptionCheck(JNIEnv* env) {
    enter(env, 1);
    return ME(env)->pending ? JNI_TRUE : JNI_FALSE;
}
static jsize JNICALL m_GetArrayLength(JNIEnv* env, jarray a) {
    enter(env, 0);
    if (!a || OBJ(a)->type < T_BYTE || OBJ(a)->type > T_DOUBLE) {
        violation(env);
        return 0;
    }
    return OBJ(a)->len;
}
static void* copy_out(JNIEnv* env, jarray a) {
    MockObj* o = OBJ(a);
    void* p = malloc((size_t)(o->len > 0 ? o->len : 1) * ELEM[o->type]);
    memcpy(p, o->data, (size_t)o->len * ELEM[o->type]);
    ME(env)->n_copies++;
    return p;
}
static void release_copy(JNIEnv* env, jarray a, void* p, jint mode) {
    MockObj* o = OBJ(a);
    if (mode == 0 || mode == JNI_COMMIT) memcpy(o->data, p, (size_t)o->len * ELEM[o->type]);
    else if (mode != JNI_ABORT) violation(env);
    if (mode != JNI_COMMIT) free(p);
}
static void* JNICALL m_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* isCopy) {
    MockEnv* e = ME(env);
    e->n_calls++;
    e->n_critical++;
    if (e->pending) e->violations++;
    if (!a || OBJ(a)->type < T_BYTE || OBJ(a)->type > T_DOUBLE) {
        violation(env);
        return NULL;
    }
    e->in_critical++;
    if (isCopy) *isCopy = JNI_TRUE;
    return copy_out(env, a);
}
static void JNICALL m_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* p, jint mode) {
    MockEnv* e = ME(env);
    e->n_calls++;
    if (e->in_critical <= 0) e->violations++;
    else e->in_critical--;
    release_copy(env, a, p, mode);
}
static jbyteArray JNICALL m_NewByteArray(JNIEnv* env, jsize len) {
    enter(env, 0);
    MockObj* o = calloc(1, sizeof *o);
    o->type = T_BYTE;
    o->len = len;
    o->data = calloc((size_t)(len > 0 ? len : 1), 1);
    return (jbyteArray)o;
}
/* <Type>ArrayRegion: type and bounds checked like the JVM */
static int region_ok(JNIEnv* env, jarray a, int type, jsize start, jsize len) {
    if (!a || OBJ(a)->type != type) {
        violation(env);
        throw_(env, "java/lang/ArrayStoreException", "mock: array type mismatch");
        return 0;
    }
    if (start < 0 || len < 0 || (int64_t)start + len > OBJ(a)->len) {
        throw_(env, "java/lang/ArrayIndexOutOfBoundsException", "mock: region out of bounds");
        return 0;
    }
    return 1;
}
#define REGION(Name, JT, TYPE)                                                                             \
    static void JNICALL m_Get##Name##ArrayRegion(JNIEnv* env, jarray a, jsize start, jsize len, JT* buf) { \
        enter(env, 0);                                                                                     \
        if (region_ok(env, a, TYPE, start, len))                                                           \
            memcpy(buf, (JT*)OBJ(a)->data + start, (size_t)len * sizeof(JT));                              \
    }
#define SET_REGION(Name, JT, TYPE)                                                                                 \
    static void JNICALL m_Set##Name##ArrayRegion(JNIEnv* env, jarray a, jsize start, jsize len, const JT* buf) { \
        enter(env, 0);                                                                                             \
        if (region_ok(env, a, TYPE, start, len))                                                                   \
            memcpy((JT*)OBJ(a)->data + start, buf, (size_t)len * sizeof(JT));                                      \
    }
REGION(Byte, jbyte, T_BYTE)
REGION(Short, jshort, T_SHORT)
REGION(Int, jint, T_INT)
REGION(Long, jlong, T_LONG)
REGION(Float, jfloat, T_FLOAT)
REGION(Double, jdouble, T_DOUBLE)
SET_REGION(Byte, jbyte, T_BYTE)
SET_REGION(Float, jfloat, T_FLOAT)
SET_REGION(Double, jdouble, T_DOUBLE)

static jfloat* JNICALL m_GetFloatArrayElements(JNIEnv* env, jfloatArray a, jboolean* isCopy) {
    enter(env, 0);
    if (!a || OBJ(a)->type != T_FLOAT) {
        violation(env);
        return NULL;
    }
    if (isCopy) *isCopy = JNI_TRUE;
    return (jfloat*)copy_out(env, a);
}
static void JNICALL m_ReleaseFloatArrayElements(JNIEnv* env, jfloatArray a, jfloat* p, jint mode) {
    ME(env)->n_calls++;
    release_copy(env, a, p, mode);
}
static const char* JNICALL m_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* isCopy) {
    enter(env, 0);
    if (!s || OBJ(s)->type != T_STRING) {
        violation(env);
        return NULL;
    }
    if (isCopy) *isCopy = JNI_TRUE;
    return strdup((const char*)OBJ(s)->data);
}
static void JNICALL m_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* chars) {
    (void)s;
    ME(env)->n_calls++;
    free((void*)chars);
}

static const struct JNINativeInterface_ g_fn = {
    .FindClass = m_FindClass,
    .ThrowNew = m_ThrowNew,
    .ExceptionCheck = m_ExceptionCheck,
    .GetArrayLength = m_GetArrayLength,
    .GetPrimitiveArrayCritical = m_GetPrimitiveArrayCritical,
    .ReleasePrimitiveArrayCritical = m_ReleasePrimitiveArrayCritical,
    .NewByteArray = m_NewByteArray,
    .GetByteArrayRegion = m_GetByteArrayRegion,
    .SetByteArrayRegion = m_SetByteArrayRegion,
    .GetShortArrayRegion = m_GetShortArrayRegion,
    .GetIntArrayRegion = m_GetIntArrayRegion,
    .GetLongArrayRegion = m_GetLongArrayRegion,
    .GetFloatArrayRegion = m_GetFloatArrayRegion,
    .SetFloatArrayRegion = m_SetFloatArrayRegion,
    .GetDoubleArrayRegion = m_GetDoubleArrayRegion,
    .SetDoubleArrayRegion = m_SetDoubleArrayRegion,
    .GetFloatArrayElements = m_GetFloatArrayElements,
    .ReleaseFloatArrayElements = m_ReleaseFloatArrayElements,
    .GetStringUTFChars = m_GetStringUTFChars,
    .ReleaseStringUTFChars = m_ReleaseStringUTFChars,
};

/* ---- the tests' side (ctypes) ---- */
__attribute__((visibility("default"))) void* mock_env_new(void) {
    MockEnv* e = calloc(1, sizeof *e);
    e->fn = &g_fn;
    return e;
}
__attribute__((visibility("default"))) void mock_env_free(void* env) { free(env); }
/* 1 if an exception is pending: its class and message are copied out, and cleared when `clear` */
__attribute__((visibility("default"))) int mock_exception(void* env, char* cls, int ncls, char* msg, int nmsg,
                                                          int clear) {
    MockEnv* e = env;
    if (!e->pending) return 0;
    if (cls) snprintf(cls, (size_t)ncls, "%s", e->exc_class);
    if (msg) snprintf(msg, (size_t)nmsg, "%s", e->exc_msg);
    if (clear) e->pending = 0;
    return 1;
}
/* calls, critical regions entered, element copies made, contract violations; and the open critical depth */
__attribute__((visibility("default"))) void mock_env_stats(void* env, long* out5) {
    MockEnv* e = env;
    out5[0] = e->n_calls;
    out5[1] = e->n_critical;
    out5[2] = e->n_copies;
    out5[3] = e->violations;
    out5[4] = e->in_critical;
}
__attribute__((visibility("default"))) void* mock_array_new(int type, int64_t len, const void* src) {
    if (type < T_BYTE || type > T_DOUBLE || len < 0 || len > INT32_MAX) return NULL;
    MockObj* o = calloc(1, sizeof *o);
    o->type = type;
    o->len = (jsize)len;
    o->data = calloc((size_t)(len > 0 ? len : 1), ELEM[type]);
    if (src && len > 0) memcpy(o->data, src, (size_t)len * ELEM[type]);
    return o;
}
__attribute__((visibility("default"))) int64_t mock_array_len(void* a) { return OBJ(a)->len; }
__attribute__((visibility("default"))) void mock_array_read(void* a, void* dst) {
    memcpy(dst, OBJ(a)->data, (size_t)OBJ(a)->len * ELEM[OBJ(a)->type]);
}
__attribute__((visibility("default"))) void* mock_string_new(const char* s) {
    MockObj* o = calloc(1, sizeof *o);
    o->type = T_STRING;
    o->data = strdup(s);
    o->len = (jsize)strlen(s);
    return o;
}
__attribute__((visibility("default"))) void mock_obj_free(void* p) {
    if (!p) return;
    free(OBJ(p)->data);
    free(p);
}
