package de.hpi.collaborativefilteringkafka.nativeals;

/**
 * JNI binding of libcfk_als.so (include/als.h, include/als_host.h) for the reference's own JDK level (Java 13,
 * build.gradle:8). The native side is integration/jni/cfk_als_jni.c (libcfk_als_jni.so, linked against
 * libcfk_als.so). Every method maps to one C entry point; a non-zero als_status is thrown by the shim as
 * org.apache.kafka.streams.errors.StreamsException carrying als_last_error(), which is what the Kafka Streams
 * runtime expects of a failing processor (the reference ignores EJML invert's boolean, MFeatureCalculator.java:98).
 *
 * Arrays are caller-owned; the shim copies them with Get/Set<Type>ArrayRegion (no JNI critical region is held while
 * a call waits on the GPU). Factor matrices are row-major float[] (double[] for ALS_F64 engines, the fp64 parity
 * mode) with a row stride of ld elements. Engine handles are als_engine* carried as long.
 * The Java 22+ alternative without a native shim is AlsFfm (Panama FFM).
 */
public final class AlsNative {
    static {
        System.loadLibrary(System.getProperty("cfk.als.jni", "cfk_als_jni"));
    }

    public static final int SIDE_MOVIE = 0, SIDE_USER = 1;
    public static final int F32 = 0, F64 = 1;
    public static final int ABI_VERSION = 3;     // include/als.h ALS_ABI_VERSION this binding was written for

    private AlsNative() {}

    /** als_abi_version */
    public static native int abiVersion();
    /** als_device_count */
    public static native int deviceCount();
    /** als_engine_create: one engine per (stream task, side); returns the als_engine* handle. */
    public static native long create(int device, int numFeatures, int precision);
    /** als_engine_destroy */
    public static native void destroy(long engine);
    /** als_set_block_coo: a partition's (local row, opposite row, rating) records in arrival order. */
    public static native void setBlockCoo(long engine, int side, long nRows, long rowOffset, long nOppRows,
                                          int[] rows, int[] cols, short[] ratings);
    /** als_alloc_factors */
    public static native void allocFactors(long engine, int side, long nRows);
    /** als_write_factors: rows [row0, row0 + rows.length / ld) from a row-major host matrix of stride ld. */
    public static native void writeFactors(long engine, int side, long row0, float[] rows, int ld);
    /** als_read_factors (synchronising: device errors surface here) */
    public static native void readFactors(long engine, int side, long row0, float[] out, int ld);
    /** als_write_factors of an F64 engine (fp64 parity mode) */
    public static native void writeFactorsF64(long engine, int side, long row0, double[] rows, int ld);
    /** als_read_factors of an F64 engine */
    public static native void readFactorsF64(long engine, int side, long row0, double[] out, int ld);
    /** als_solve_half: THE HOT PATH, every row of the side's block (MFeatureCalculator.java:66-104), asynchronous. */
    public static native void solveHalf(long engine, int side, float lambda);
    /** als_synchronize */
    public static native void synchronize(long engine);
    /** als_comm_unique_id: the 128-byte RCCL unique id (rank 0 of a G-GPU job). */
    public static native byte[] commUniqueId();
    /** als_comm_init: this engine becomes rank `rank` of `world`. */
    public static native void commInit(long engine, int world, int rank, byte[] uniqueId);
    /** als_comm_set_timeout: bound on every wait for this engine's exchanges (ms); past it the communicator is
     *  aborted and the waiting call throws, naming the pending all-gather. */
    public static native void commSetTimeout(long engine, long timeoutMs);
    /** als_allgather_shard: chunk `chunk` of the side's chunk-major slots (unchunked: slotsPerShard, 0). */
    public static native void allgatherShard(long engine, int side, long slotsPerChunk, long chunk);
    /** als_predict: out[u * movieRows.length + m] = U[userRows[u]] . M[movieRows[m]] as a Java float dot. */
    public static native void predict(long engine, long[] userRows, long[] movieRows, float[] out);
    /** als_write_prediction_matrix_csv: EJML saveDenseCSV layout (FeatureCollector.java:103-106). */
    public static native void writePredictionMatrixCsv(String path, float[] prediction, long nUsers, long nMovies);
}
