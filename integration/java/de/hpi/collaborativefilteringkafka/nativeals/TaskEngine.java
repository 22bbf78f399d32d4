package de.hpi.collaborativefilteringkafka.nativeals;

import de.hpi.collaborativefilteringkafka.apps.ALSApp;
import org.apache.kafka.streams.processor.TaskId;
import org.apache.kafka.streams.state.KeyValueIterator;
import org.apache.kafka.streams.state.KeyValueStore;

import java.util.ArrayList;
import java.util.Arrays;
import java.util.HashMap;

/**
 * One GPU engine per (stream task, side), shared by that task's NUM_ALS_ITERATIONS calculator instances.
 *
 * The reference unrolls the ALS loop into one MFeatureCalculator-i / UFeatureCalculator-i processor per iteration
 * (ALSApp.java:115-151); all of them sit in the same sub-topology and read the same in-block stores, so Kafka
 * Streams gives one task (partition p) all N instances. They share this object: the in-blocks are uploaded to the
 * device ONCE per task and side (they never change, README.md:146-147), not once per processor instance.
 * A task is processed by one stream thread at a time (BaseKafkaApp.java:51: 4 threads over 2P+1 tasks), so only
 * the registry needs a lock.
 *
 * Readiness. The reference solves an entity as soon as all of its in-block rows arrived (MFeatureCalculator.java:65).
 * Every opposite entity that appears in this partition's in-blocks sends exactly one FeatureMessage to this
 * partition per half (the out-block fan-out, MFeatureCalculator.java:125-131 / UFeatureCalculator.java:124-131),
 * so the partition's half is complete when every distinct opposite id of its in-blocks has arrived for that
 * iteration. Rows are staged per iteration (the source topic), which keeps a fast upstream task's next-iteration
 * rows apart. Then the whole half is ONE als_solve_half call (AlsNative.solveHalf).
 */
public final class TaskEngine {
    private static final HashMap<String, TaskEngine> REGISTRY = new HashMap<>();

    private final String key;
    private final int side;                  // AlsNative.SIDE_MOVIE: solves movies from user rows
    private final long engine;
    private int refs;

    private int[] rowIds;                    // local row -> entity id (ascending: the collector's order)
    private HashMap<Integer, Integer> oppSlot;   // opposite id -> row of the engine's opposite replica
    private final HashMap<Integer, float[]> staged = new HashMap<>();      // iteration -> opposite rows x k
    private final HashMap<Integer, boolean[]> seen = new HashMap<>();
    private final HashMap<Integer, Integer> arrived = new HashMap<>();

    private TaskEngine(String key, int side, int device) {
        this.key = key;
        this.side = side;
        this.engine = AlsNative.create(device, ALSApp.NUM_FEATURES, AlsNative.F32);
    }

    /**
     * The engine of (task, side), created on first use on GPU task.partition % cfk.gpus (one engine per GPU when
     * the task count equals the GPU count). TaskId.partition is valid in init(); ProcessorContext.partition() is
     * not (it names the partition of the record being processed, kafka-streams 2.3.1).
     */
    public static TaskEngine acquire(TaskId task, int side) {
        synchronized (REGISTRY) {
            final String key = task.toString() + "/" + side;
            TaskEngine e = REGISTRY.get(key);
            if (e == null) {
                final int gpus = Math.max(1, Integer.getInteger("cfk.gpus", AlsNative.deviceCount()));
                e = new TaskEngine(key, side, task.partition % gpus);
                REGISTRY.put(key, e);
            }
            e.refs++;
            return e;
        }
    }

    /** Drops one processor's reference; the last one destroys the engine (Processor.close). */
    public void release() {
        synchronized (REGISTRY) {
            if (--refs == 0) {
                REGISTRY.remove(key);
                AlsNative.destroy(engine);
            }
        }
    }

    /** Entity ids of the block's rows, ascending (row r of solve()'s result). */
    public int[] rowIds() {
        return rowIds;
    }

    /**
     * Uploads this task's in-blocks (inIds / inRatings: the stores MRatings2BlocksProcessor.java:48-69 resp.
     * URatings2BlocksProcessor.java:72-92 filled before the EOF barrier) on the first call; later calls return.
     */
    public void ensureBlocks(KeyValueStore<Integer, ArrayList<Integer>> inIds,
                             KeyValueStore<Integer, ArrayList<Short>> inRatings) {
        if (rowIds != null) return;
        final ArrayList<Integer> ids = new ArrayList<>();
        try (KeyValueIterator<Integer, ArrayList<Integer>> it = inIds.all()) {
            it.forEachRemaining(kv -> ids.add(kv.key));
        }
        final int[] rows = ids.stream().mapToInt(Integer::intValue).sorted().toArray();
        final HashMap<Integer, Integer> slots = new HashMap<>();
        int nnz = 0;
        for (int id : rows) nnz += inIds.get(id).size();
        final int[] r = new int[nnz], c = new int[nnz];
        final short[] v = new short[nnz];
        int t = 0;
        for (int i = 0; i < rows.length; i++) {
            final ArrayList<Integer> opp = inIds.get(rows[i]);
            final ArrayList<Short> ratings = inRatings.get(rows[i]);
            for (int q = 0; q < opp.size(); q++, t++) {   // in-block order = arrival order
                r[t] = i;
                c[t] = slots.computeIfAbsent(opp.get(q), o -> slots.size());
                v[t] = ratings.get(q);
            }
        }
        AlsNative.allocFactors(engine, 1 - side, slots.size());
        AlsNative.allocFactors(engine, side, rows.length);
        AlsNative.setBlockCoo(engine, side, rows.length, 0, slots.size(), r, c, v);
        rowIds = rows;
        oppSlot = slots;
    }

    /** Stages one opposite row of `iteration`; true when it completes the half (every opposite id arrived). */
    public boolean stage(int iteration, int oppId, float[] features) {
        final Integer slot = oppSlot.get(oppId);
        if (slot == null) return false;              // no entity of this partition depends on it
        final int k = ALSApp.NUM_FEATURES;
        final float[] rows = staged.computeIfAbsent(iteration, i -> new float[oppSlot.size() * k]);
        final boolean[] s = seen.computeIfAbsent(iteration, i -> new boolean[oppSlot.size()]);
        System.arraycopy(features, 0, rows, slot * k, k);
        if (!s[slot]) {
            s[slot] = true;
            arrived.merge(iteration, 1, Integer::sum);
        }
        return arrived.get(iteration) == oppSlot.size();
    }

    /**
     * The half of `iteration`: one upload of the staged opposite replica, ONE als_solve_half over every row of the
     * partition (MFeatureCalculator.java:66-104 / UFeatureCalculator.java:66-104 for all entities at once), one
     * read-back (synchronising: any device error is thrown here). Returns row r's features at [r k, (r+1) k).
     */
    public float[] solve(int iteration, float lambda) {
        final int k = ALSApp.NUM_FEATURES;
        AlsNative.writeFactors(engine, 1 - side, 0, staged.remove(iteration), k);
        seen.remove(iteration);
        arrived.remove(iteration);
        AlsNative.solveHalf(engine, side, lambda);
        final float[] out = new float[rowIds.length * k];
        AlsNative.readFactors(engine, side, 0, out, k);
        return out;
    }

    /** Row r of a solve() result as the reference's float[] message payload. */
    public static float[] row(float[] solved, int r) {
        final int k = ALSApp.NUM_FEATURES;
        return Arrays.copyOfRange(solved, r * k, (r + 1) * k);
    }
}
