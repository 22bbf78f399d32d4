package de.hpi.collaborativefilteringkafka.nativeals;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_FLOAT;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Panama FFM (Java 22+) binding of libcfk_als.so, the C ABI declared in include/als.h (the processors under
 * processors/ use the JNI binding AlsNative, which runs on the reference's Java 13). No native shim: every
 * downcall handle below binds one exported symbol with the descriptor of its C prototype
 * (int -> JAVA_INT, int64_t -> JAVA_LONG, float -> JAVA_FLOAT, any pointer -> ADDRESS).
 * tests/test_integration_java.py checks each descriptor against the library's ctypes signatures.
 *
 * Replaces the EJML calls of the reference's hot path (processors/MFeatureCalculator.java:85-99,
 * processors/UFeatureCalculator.java:85-99). Status codes become exceptions on the Java side, as the
 * Kafka Streams runtime expects of a processor (the reference ignores invert()'s boolean, :98).
 */
public final class AlsFfm {
    public static final int SIDE_MOVIE = 0, SIDE_USER = 1;
    public static final int F32 = 0, F64 = 1;
    public static final int ALS_OK = 0;

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("cfk.als.lib", "libcfk_als.so"), Arena.global());

    private static MethodHandle h(String name, FunctionDescriptor d) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
                () -> new UnsatisfiedLinkError("libcfk_als.so does not export " + name)), d);
    }

    // ---- version / errors (als.h:57-59)
    static final MethodHandle ABI_VERSION = h("als_abi_version", FunctionDescriptor.of(JAVA_INT));
    static final MethodHandle LAST_ERROR = h("als_last_error", FunctionDescriptor.of(ADDRESS));
    static final MethodHandle DEVICE_COUNT = h("als_device_count", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // ---- engine lifetime (als.h:64-75)
    static final MethodHandle ENGINE_CREATE = h("als_engine_create",
            FunctionDescriptor.of(JAVA_INT, JAVA_INT, JAVA_INT, JAVA_INT, ADDRESS));
    static final MethodHandle ENGINE_DESTROY = h("als_engine_destroy", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    static final MethodHandle ENGINE_SET_STREAM = h("als_engine_set_stream",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle FACTOR_STRIDE = h("als_factor_stride", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // ---- in-blocks (als.h:83-91)
    static final MethodHandle SET_BLOCK = h("als_set_block", FunctionDescriptor.of(JAVA_INT,
            ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SET_BLOCK_COO = h("als_set_block_coo", FunctionDescriptor.of(JAVA_INT,
            ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS, ADDRESS));
    // ---- factor matrices (als.h:96-106)
    static final MethodHandle ALLOC_FACTORS = h("als_alloc_factors",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG));
    static final MethodHandle WRITE_FACTORS = h("als_write_factors",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG, ADDRESS, JAVA_LONG));
    static final MethodHandle READ_FACTORS = h("als_read_factors",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG, ADDRESS, JAVA_LONG));
    // ---- the hot path (als.h:113-123)
    static final MethodHandle SOLVE_HALF = h("als_solve_half",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_FLOAT));
    static final MethodHandle SET_CHUNKS = h("als_set_chunks",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
    static final MethodHandle SOLVE_HALF_CHUNK = h("als_solve_half_chunk",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_FLOAT, JAVA_INT));
    // ---- multi-GPU exchange (als.h:132-146)
    static final MethodHandle COMM_UNIQUE_ID = h("als_comm_unique_id",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
    static final MethodHandle COMM_INIT = h("als_comm_init",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, ADDRESS));
    static final MethodHandle ALLGATHER_SHARD = h("als_allgather_shard",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG));
    static final MethodHandle SET_ROW_LAYOUT = h("als_set_row_layout",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_LONG, JAVA_LONG));
    static final MethodHandle COMM_WAIT = h("als_comm_wait", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // ---- collector, MSE, synchronisation (als.h:153-166)
    static final MethodHandle PREDICT = h("als_predict",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle SQ_ERROR = h("als_sq_error",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, ADDRESS));
    static final MethodHandle SYNCHRONIZE = h("als_synchronize", FunctionDescriptor.of(JAVA_INT, ADDRESS));
    // ---- host layer (als_host.h): the collector's CSV writer
    static final MethodHandle WRITE_PREDICTION_MATRIX_CSV = h("als_write_prediction_matrix_csv",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG));

    private AlsFfm() {}

    /** A non-zero als_status as an exception carrying als_last_error() (the calling thread's message). */
    public static final class AlsException extends RuntimeException {
        public final int status;
        AlsException(String fn, int status, String msg) {
            super(fn + ": status " + status + ": " + msg);
            this.status = status;
        }
    }

    static void check(String fn, Object status) {
        int st = (Integer) status;
        if (st != ALS_OK) {
            String msg;
            try {
                MemorySegment p = (MemorySegment) LAST_ERROR.invokeExact();
                msg = p.reinterpret(4096).getString(0);
            } catch (Throwable t) {
                msg = "(als_last_error unavailable: " + t + ")";
            }
            throw new AlsException(fn, st, msg);
        }
    }

    static RuntimeException rethrow(Throwable t) {
        return t instanceof RuntimeException ? (RuntimeException) t : new RuntimeException(t);
    }

    /** als_engine_create: one engine per stream task / GPU (MFeatureCalculator.init, :29-46). */
    public static MemorySegment createEngine(int device, int numFeatures, int precision) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(ADDRESS);
            check("als_engine_create", (int) ENGINE_CREATE.invokeExact(device, numFeatures, precision, out));
            return out.get(ADDRESS, 0);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static void destroyEngine(MemorySegment e) {
        try {
            check("als_engine_destroy", (int) ENGINE_DESTROY.invokeExact(e));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** als_set_block_coo: the partition's (local row, opposite row, rating) records in arrival order. */
    public static void setBlockCoo(MemorySegment e, int side, long nRows, long rowOffset, long nOppRows,
                                   int[] rows, int[] cols, short[] ratings) {
        try (Arena a = Arena.ofConfined()) {
            check("als_set_block_coo", (int) SET_BLOCK_COO.invokeExact(e, side, nRows, rowOffset, nOppRows,
                    (long) rows.length, a.allocateFrom(JAVA_INT, rows), a.allocateFrom(JAVA_INT, cols),
                    a.allocateFrom(java.lang.foreign.ValueLayout.JAVA_SHORT, ratings)));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static void allocFactors(MemorySegment e, int side, long nRows) {
        try {
            check("als_alloc_factors", (int) ALLOC_FACTORS.invokeExact(e, side, nRows));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** Rows [row0, row0 + rows.length / ld) of `side` from a host row-major float matrix of row stride ld. */
    public static void writeFactors(MemorySegment e, int side, long row0, float[] rows, int ld) {
        try (Arena a = Arena.ofConfined()) {
            check("als_write_factors", (int) WRITE_FACTORS.invokeExact(e, side, row0, (long) (rows.length / ld),
                    a.allocateFrom(JAVA_FLOAT, rows), (long) ld));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static void readFactors(MemorySegment e, int side, long row0, float[] out, int ld) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment dst = a.allocate(JAVA_FLOAT, out.length);
            check("als_read_factors", (int) READ_FACTORS.invokeExact(e, side, row0, (long) (out.length / ld),
                    dst, (long) ld));
            MemorySegment.copy(dst, JAVA_FLOAT, 0, out, 0, out.length);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** THE HOT PATH: every row of `side` in one call (MFeatureCalculator.java:66-104 for the whole partition). */
    public static void solveHalf(MemorySegment e, int side, float lambda) {
        try {
            check("als_solve_half", (int) SOLVE_HALF.invokeExact(e, side, lambda));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static byte[] commUniqueId() {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment id = a.allocate(128);
            check("als_comm_unique_id", (int) COMM_UNIQUE_ID.invokeExact(id, 128));
            return id.toArray(java.lang.foreign.ValueLayout.JAVA_BYTE);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static void commInit(MemorySegment e, int world, int rank, byte[] uniqueId) {
        try (Arena a = Arena.ofConfined()) {
            check("als_comm_init", (int) COMM_INIT.invokeExact(e, world, rank,
                    a.allocateFrom(java.lang.foreign.ValueLayout.JAVA_BYTE, uniqueId)));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** Chunk `chunk` of the side's chunk-major slots (an unchunked side: its slots per shard, chunk 0). */
    public static void allgatherShard(MemorySegment e, int side, long slotsPerChunk, long chunk) {
        try {
            check("als_allgather_shard", (int) ALLGATHER_SHARD.invokeExact(e, side, slotsPerChunk, chunk));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** Local row i -> factor row rowOffset + (i / rowsPerChunk) * chunkStride + i % rowsPerChunk. */
    public static void setRowLayout(MemorySegment e, int side, long rowsPerChunk, long chunkStride) {
        try {
            check("als_set_row_layout", (int) SET_ROW_LAYOUT.invokeExact(e, side, rowsPerChunk, chunkStride));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    /** FeatureCollector.calculatePredictionMatrix (FeatureCollector.java:90-101) on the resident factors. */
    public static float[] predict(MemorySegment e, long[] userRows, long[] movieRows) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_FLOAT, (long) userRows.length * movieRows.length);
            check("als_predict", (int) PREDICT.invokeExact(e, a.allocateFrom(JAVA_LONG, userRows),
                    (long) userRows.length, a.allocateFrom(JAVA_LONG, movieRows), (long) movieRows.length, out));
            return out.toArray(JAVA_FLOAT);
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }

    public static void synchronize(MemorySegment e) {
        try {
            check("als_synchronize", (int) SYNCHRONIZE.invokeExact(e));
        } catch (Throwable t) {
            throw rethrow(t);
        }
    }
}
