/*
 * cfk_als_jni.c -- JNI shim between de.hpi.collaborativefilteringkafka.nativeals.AlsNative (Java 13, the
 * reference's level: build.gradle:8) and the C ABI of libcfk_als.so (include/als.h, include/als_host.h).
 *
 *   gcc -O2 -shared -fPIC -I"$JAVA_HOME/include" -I"$JAVA_HOME/include/linux" -I include \
 *       integration/jni/cfk_als_jni.c -o libcfk_als_jni.so \
 *       -L collaborative-filtering-kafka_amd/build -lcfk_als -Wl,-rpath,'$ORIGIN'
 *
 * (integration/jni/Makefile.) There is no JDK in the build image: tests/jni compiles this same file against a
 * test-only jni.h and drives every entry point through a mock JVM (tests/test_jni_shim.py), including 8 engines
 * called from 4 threads on the GPU.
 *
 * Every native method forwards to one C entry point. Arrays cross with Get/Set<Type>ArrayRegion into native buffers:
 * the calls behind them wait on the GPU (als_set_block_coo builds the block on the device, als_write_factors /
 * als_read_factors / als_predict synchronise), and a JNI critical region held that long would stall the garbage
 * collector for the other stream threads (GCLocker). A non-zero als_status becomes a StreamsException carrying
 * als_last_error(): a failing processor then stops its stream thread exactly as an exception inside the
 * reference's process() would (kafka-streams 2.3.1 default handler).
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "als.h"
#include "als_host.h"

#define ENGINE(h) ((als_engine*)(intptr_t)(h))

/* Throws (pending Java exception) and returns non-zero when status is an error. */
static int fail_status(JNIEnv* env, const char* fn, int status) {
    if (status == ALS_OK) return 0;
    char msg[1024];
    snprintf(msg, sizeof msg, "%s: als_status %d: %s", fn, status, als_last_error());
    jclass ex = (*env)->FindClass(env, "org/apache/kafka/streams/errors/StreamsException");
    if (ex == NULL) ex = (*env)->FindClass(env, "java/lang/RuntimeException");
    if (ex != NULL) (*env)->ThrowNew(env, ex, msg);
    return 1;
}

static int fail_arg(JNIEnv* env, const char* what) {
    jclass ex = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
    if (ex != NULL) (*env)->ThrowNew(env, ex, what);
    return 1;
}

static int fail_oom(JNIEnv* env, const char* what) {
    jclass ex = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (ex != NULL) (*env)->ThrowNew(env, ex, what);
    return 1;
}

/* malloc of n elements of `size` bytes (n may be 0: returns a valid pointer) */
static void* alloc_n(JNIEnv* env, jsize n, size_t size, const char* what) {
    void* p = malloc((size_t)(n > 0 ? n : 1) * size);
    if (p == NULL) fail_oom(env, what);
    return p;
}

JNIEXPORT jint JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_abiVersion(JNIEnv* env,
                                                                                             jclass cls) {
    (void)env;
    (void)cls;
    return als_abi_version();
}

JNIEXPORT jint JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_deviceCount(JNIEnv* env,
                                                                                              jclass cls) {
    (void)cls;
    int n = 0;
    fail_status(env, "als_device_count", als_device_count(&n));
    return n;
}

JNIEXPORT jlong JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_create(
        JNIEnv* env, jclass cls, jint device, jint num_features, jint precision) {
    (void)cls;
    als_engine* e = NULL;
    if (fail_status(env, "als_engine_create", als_engine_create(device, num_features, precision, &e))) return 0;
    return (jlong)(intptr_t)e;
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_destroy(JNIEnv* env, jclass cls,
                                                                                          jlong engine) {
    (void)cls;
    fail_status(env, "als_engine_destroy", als_engine_destroy(ENGINE(engine)));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_setBlockCoo(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong n_rows, jlong row_offset, jlong n_opp_rows,
        jintArray rows, jintArray cols, jshortArray ratings) {
    (void)cls;
    const jsize nnz = (*env)->GetArrayLength(env, rows);
    if ((*env)->GetArrayLength(env, cols) != nnz || (*env)->GetArrayLength(env, ratings) != nnz) {
        fail_arg(env, "setBlockCoo: rows, cols and ratings differ in length");
        return;
    }
    jint* r = alloc_n(env, nnz, sizeof(jint), "setBlockCoo: rows");
    jint* c = r ? alloc_n(env, nnz, sizeof(jint), "setBlockCoo: cols") : NULL;
    jshort* v = c ? alloc_n(env, nnz, sizeof(jshort), "setBlockCoo: ratings") : NULL;
    if (v != NULL) {
        (*env)->GetIntArrayRegion(env, rows, 0, nnz, r);
        (*env)->GetIntArrayRegion(env, cols, 0, nnz, c);
        (*env)->GetShortArrayRegion(env, ratings, 0, nnz, v);
        if (!(*env)->ExceptionCheck(env))
            fail_status(env, "als_set_block_coo",
                        als_set_block_coo(ENGINE(engine), side, n_rows, row_offset, n_opp_rows, nnz,
                                          (const int32_t*)r, (const int32_t*)c, (const int16_t*)v));
    }
    free(v);
    free(c);
    free(r);
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_allocFactors(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong n_rows) {
    (void)cls;
    fail_status(env, "als_alloc_factors", als_alloc_factors(ENGINE(engine), side, n_rows));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_writeFactors(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong row0, jfloatArray rows, jint ld) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, rows);
    if (ld <= 0 || n % ld != 0) {
        fail_arg(env, "writeFactors: rows.length must be a multiple of ld");
        return;
    }
    jfloat* p = alloc_n(env, n, sizeof(jfloat), "writeFactors");
    if (p == NULL) return;
    (*env)->GetFloatArrayRegion(env, rows, 0, n, p);
    if (!(*env)->ExceptionCheck(env))
        fail_status(env, "als_write_factors", als_write_factors(ENGINE(engine), side, row0, n / ld, p, ld));
    free(p);
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_readFactors(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong row0, jfloatArray out, jint ld) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, out);
    if (ld <= 0 || n % ld != 0) {
        fail_arg(env, "readFactors: out.length must be a multiple of ld");
        return;
    }
    jfloat* p = alloc_n(env, n, sizeof(jfloat), "readFactors");
    if (p == NULL) return;
    /* als_read_factors writes the first num_features of each ld-strided row: the rest of the buffer starts as the
     * Java array's own contents, so the whole-array copy back leaves those columns as they were */
    (*env)->GetFloatArrayRegion(env, out, 0, n, p);
    if (!(*env)->ExceptionCheck(env) &&
        !fail_status(env, "als_read_factors", als_read_factors(ENGINE(engine), side, row0, n / ld, p, ld)))
        (*env)->SetFloatArrayRegion(env, out, 0, n, p);
    free(p);
}

/* fp64 parity mode (ALS_F64 engines): the same copies with double[] (als_write_factors / als_read_factors take the
 * engine's element type) */
JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_writeFactorsF64(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong row0, jdoubleArray rows, jint ld) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, rows);
    if (ld <= 0 || n % ld != 0) {
        fail_arg(env, "writeFactorsF64: rows.length must be a multiple of ld");
        return;
    }
    jdouble* p = alloc_n(env, n, sizeof(jdouble), "writeFactorsF64");
    if (p == NULL) return;
    (*env)->GetDoubleArrayRegion(env, rows, 0, n, p);
    if (!(*env)->ExceptionCheck(env))
        fail_status(env, "als_write_factors", als_write_factors(ENGINE(engine), side, row0, n / ld, p, ld));
    free(p);
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_readFactorsF64(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong row0, jdoubleArray out, jint ld) {
    (void)cls;
    const jsize n = (*env)->GetArrayLength(env, out);
    if (ld <= 0 || n % ld != 0) {
        fail_arg(env, "readFactorsF64: out.length must be a multiple of ld");
        return;
    }
    jdouble* p = alloc_n(env, n, sizeof(jdouble), "readFactorsF64");
    if (p == NULL) return;
    (*env)->GetDoubleArrayRegion(env, out, 0, n, p);   /* untouched columns round-trip (as readFactors) */
    if (!(*env)->ExceptionCheck(env) &&
        !fail_status(env, "als_read_factors", als_read_factors(ENGINE(engine), side, row0, n / ld, p, ld)))
        (*env)->SetDoubleArrayRegion(env, out, 0, n, p);
    free(p);
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_solveHalf(
        JNIEnv* env, jclass cls, jlong engine, jint side, jfloat lambda) {
    (void)cls;
    fail_status(env, "als_solve_half", als_solve_half(ENGINE(engine), side, lambda));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_synchronize(JNIEnv* env,
                                                                                              jclass cls,
                                                                                              jlong engine) {
    (void)cls;
    fail_status(env, "als_synchronize", als_synchronize(ENGINE(engine)));
}

JNIEXPORT jbyteArray JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_commUniqueId(JNIEnv* env,
                                                                                                     jclass cls) {
    (void)cls;
    char id[128];
    if (fail_status(env, "als_comm_unique_id", als_comm_unique_id(id, (int)sizeof id))) return NULL;
    jbyteArray out = (*env)->NewByteArray(env, (jsize)sizeof id);
    if (out != NULL) (*env)->SetByteArrayRegion(env, out, 0, (jsize)sizeof id, (const jbyte*)id);
    return out;
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_commInit(
        JNIEnv* env, jclass cls, jlong engine, jint world, jint rank, jbyteArray unique_id) {
    (void)cls;
    jbyte buf[128];
    if ((*env)->GetArrayLength(env, unique_id) != (jsize)sizeof buf) {
        fail_arg(env, "commInit: the unique id has 128 bytes");
        return;
    }
    (*env)->GetByteArrayRegion(env, unique_id, 0, (jsize)sizeof buf, buf);
    if (!(*env)->ExceptionCheck(env))
        fail_status(env, "als_comm_init", als_comm_init(ENGINE(engine), world, rank, buf));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_commSetTimeout(
        JNIEnv* env, jclass cls, jlong engine, jlong timeout_ms) {
    (void)cls;
    fail_status(env, "als_comm_set_timeout", als_comm_set_timeout(ENGINE(engine), (int64_t)timeout_ms));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_allgatherShard(
        JNIEnv* env, jclass cls, jlong engine, jint side, jlong slots_per_chunk, jlong chunk) {
    (void)cls;
    fail_status(env, "als_allgather_shard", als_allgather_shard(ENGINE(engine), side, slots_per_chunk, chunk));
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_predict(
        JNIEnv* env, jclass cls, jlong engine, jlongArray user_rows, jlongArray movie_rows, jfloatArray out) {
    (void)cls;
    const jsize nu = (*env)->GetArrayLength(env, user_rows), nm = (*env)->GetArrayLength(env, movie_rows);
    const jsize no = (*env)->GetArrayLength(env, out);
    if ((int64_t)no != (int64_t)nu * (int64_t)nm) {
        fail_arg(env, "predict: out.length must be userRows.length * movieRows.length");
        return;
    }
    jlong* u = alloc_n(env, nu, sizeof(jlong), "predict: userRows");
    jlong* m = u ? alloc_n(env, nm, sizeof(jlong), "predict: movieRows") : NULL;
    jfloat* p = m ? alloc_n(env, no, sizeof(jfloat), "predict: out") : NULL;
    if (p != NULL) {
        (*env)->GetLongArrayRegion(env, user_rows, 0, nu, u);
        (*env)->GetLongArrayRegion(env, movie_rows, 0, nm, m);
        if (!(*env)->ExceptionCheck(env) &&
            !fail_status(env, "als_predict",
                         als_predict(ENGINE(engine), (const int64_t*)u, nu, (const int64_t*)m, nm, p)))
            (*env)->SetFloatArrayRegion(env, out, 0, no, p);
    }
    free(p);
    free(m);
    free(u);
}

JNIEXPORT void JNICALL Java_de_hpi_collaborativefilteringkafka_nativeals_AlsNative_writePredictionMatrixCsv(
        JNIEnv* env, jclass cls, jstring path, jfloatArray prediction, jlong n_users, jlong n_movies) {
    (void)cls;
    if ((int64_t)(*env)->GetArrayLength(env, prediction) != (int64_t)n_users * (int64_t)n_movies) {
        fail_arg(env, "writePredictionMatrixCsv: prediction.length must be nUsers * nMovies");
        return;
    }
    const char* cpath = (*env)->GetStringUTFChars(env, path, NULL);
    if (cpath == NULL) return;   /* OutOfMemoryError pending */
    jfloat* p = (*env)->GetFloatArrayElements(env, prediction, NULL);   /* not critical: the writer does file I/O */
    const int st = p ? als_write_prediction_matrix_csv(cpath, p, n_users, n_movies) : ALS_ERR_OUT_OF_MEMORY;
    if (p) (*env)->ReleaseFloatArrayElements(env, prediction, p, JNI_ABORT);
    (*env)->ReleaseStringUTFChars(env, path, cpath);
    fail_status(env, "als_write_prediction_matrix_csv", st);
}
