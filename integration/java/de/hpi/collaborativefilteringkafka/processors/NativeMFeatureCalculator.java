package de.hpi.collaborativefilteringkafka.processors;

import de.hpi.collaborativefilteringkafka.apps.ALSApp;
import de.hpi.collaborativefilteringkafka.messages.FeatureMessage;
import de.hpi.collaborativefilteringkafka.nativeals.AlsFfm;
import org.apache.kafka.streams.processor.AbstractProcessor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.To;
import org.apache.kafka.streams.state.KeyValueIterator;
import org.apache.kafka.streams.state.KeyValueStore;

import java.lang.foreign.MemorySegment;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.HashMap;
import java.util.stream.Collectors;

/**
 * Drop-in replacement of processors/MFeatureCalculator.java (same stores, same input and output records) that
 * solves the partition's whole movie half on the GPU with ONE AlsFfm.solveHalf call instead of one EJML solve per
 * movie (MFeatureCalculator.java:66-104). UFeatureCalculator is the same class with the sides swapped
 * (u-inblocks-mid / u-inblocks-ratings / u-outblocks, SIDE_USER, USER_FEATURES_SINK).
 *
 * Readiness: the reference solves a movie once all its users' rows arrived (:65). Every user of this partition's
 * in-blocks sends exactly one FeatureMessage per half (the out-block fan-out, :125-132 of the opposite
 * processor), so the half is complete when every distinct user of the partition has arrived; the rows are
 * staged per iteration (source topic), which also keeps a fast upstream's next-iteration rows apart.
 * Output: per movie, the same FeatureMessage records with the same dependent-id filtering and sinks (:106-132).
 */
public class NativeMFeatureCalculator extends AbstractProcessor<Integer, FeatureMessage> {
    private ProcessorContext context;
    private KeyValueStore<Integer, ArrayList<Integer>> mInBlocksUidStore;
    private KeyValueStore<Integer, ArrayList<Short>> mInBlocksRatingsStore;
    private KeyValueStore<Integer, ArrayList<Short>> mOutBlocksStore;

    private MemorySegment engine;                 // one engine per stream task (als_engine_create)
    private int[] movieIds;                        // local row -> movie id (ascending: the collector's order)
    private HashMap<Integer, Integer> userSlot;    // user id -> row of the engine's user replica
    private final HashMap<Integer, float[]> stagedRows = new HashMap<>();   // iteration -> users x k
    private final HashMap<Integer, Integer> arrived = new HashMap<>();      // iteration -> distinct users so far
    private final HashMap<Integer, boolean[]> seen = new HashMap<>();

    @Override
    @SuppressWarnings("unchecked")
    public void init(final ProcessorContext context) {
        this.context = context;
        this.mInBlocksUidStore = (KeyValueStore<Integer, ArrayList<Integer>>) context.getStateStore(ALSApp.M_INBLOCKS_UID_STORE);
        this.mInBlocksRatingsStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.M_INBLOCKS_RATINGS_STORE);
        this.mOutBlocksStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.M_OUTBLOCKS_STORE);
        // device = stream task's partition modulo the visible GPUs (one engine per GPU when tasks == GPUs)
        this.engine = AlsFfm.createEngine(context.partition() % Math.max(1, Integer.getInteger("cfk.gpus", 1)),
                ALSApp.NUM_FEATURES, AlsFfm.F32);
    }

    /** Uploads the in-blocks once (they never change, README.md:146-147) after the EOF barrier filled the stores. */
    private void buildBlocks() {
        ArrayList<Integer> ids = new ArrayList<>();
        try (KeyValueIterator<Integer, ArrayList<Integer>> it = mInBlocksUidStore.all()) {
            it.forEachRemaining(kv -> ids.add(kv.key));
        }
        movieIds = ids.stream().mapToInt(Integer::intValue).sorted().toArray();
        userSlot = new HashMap<>();
        int nnz = 0;
        for (int m : movieIds) nnz += mInBlocksUidStore.get(m).size();
        int[] rows = new int[nnz], cols = new int[nnz];
        short[] ratings = new short[nnz];
        int t = 0;
        for (int r = 0; r < movieIds.length; r++) {
            ArrayList<Integer> uids = mInBlocksUidStore.get(movieIds[r]);
            ArrayList<Short> rs = mInBlocksRatingsStore.get(movieIds[r]);
            for (int q = 0; q < uids.size(); q++, t++) {       // in-block order = arrival order (:53-69 of the builder)
                rows[t] = r;
                cols[t] = userSlot.computeIfAbsent(uids.get(q), u -> userSlot.size());
                ratings[t] = rs.get(q);
            }
        }
        AlsFfm.allocFactors(engine, AlsFfm.SIDE_USER, userSlot.size());
        AlsFfm.allocFactors(engine, AlsFfm.SIDE_MOVIE, movieIds.length);
        AlsFfm.setBlockCoo(engine, AlsFfm.SIDE_MOVIE, movieIds.length, 0, userSlot.size(), rows, cols, ratings);
    }

    @Override
    public void process(final Integer partition, final FeatureMessage msg) {
        if (movieIds == null) buildBlocks();
        final int k = ALSApp.NUM_FEATURES;
        final String sourceTopic = context.topic();
        final int iteration = Integer.parseInt(sourceTopic.substring(sourceTopic.length() - 1));   // as :106-107

        Integer slot = userSlot.get(msg.id);
        if (slot == null) return;                       // no movie of this partition depends on this user
        float[] staged = stagedRows.computeIfAbsent(iteration, i -> new float[userSlot.size() * k]);
        boolean[] s = seen.computeIfAbsent(iteration, i -> new boolean[userSlot.size()]);
        System.arraycopy(msg.features, 0, staged, slot * k, k);
        if (!s[slot]) {
            s[slot] = true;
            arrived.merge(iteration, 1, Integer::sum);
        }
        if (arrived.get(iteration) < userSlot.size()) return;

        // the whole half: one upload of the user replica, one solve of every movie of the partition, one readback
        AlsFfm.writeFactors(engine, AlsFfm.SIDE_USER, 0, staged, k);
        AlsFfm.solveHalf(engine, AlsFfm.SIDE_MOVIE, ALSApp.ALS_LAMBDA);
        float[] solved = new float[movieIds.length * k];
        AlsFfm.readFactors(engine, AlsFfm.SIDE_MOVIE, 0, solved, k);   // synchronising: throws on any device error
        stagedRows.remove(iteration);
        seen.remove(iteration);
        arrived.remove(iteration);

        for (int r = 0; r < movieIds.length; r++) {     // unchanged fan-out, MFeatureCalculator.java:106-132
            final int movieId = movieIds[r];
            float[] features = Arrays.copyOfRange(solved, r * k, (r + 1) * k);
            ArrayList<Integer> dependentUids = mInBlocksUidStore.get(movieId);
            FeatureMessage out = new FeatureMessage(movieId, dependentUids, features);
            if (iteration == ALSApp.NUM_ALS_ITERATIONS - 1) {
                context.forward(0, out, To.child(ALSApp.MOVIE_FEATURES_SINK + ALSApp.NUM_ALS_ITERATIONS));
            }
            for (int targetPartition : mOutBlocksStore.get(movieId)) {
                out.setDependentIds((ArrayList<Integer>) dependentUids.stream()
                        .filter(id -> (id % ALSApp.NUM_PARTITIONS) == targetPartition)
                        .collect(Collectors.toCollection(ArrayList::new)));
                context.forward(targetPartition, out, To.child(ALSApp.MOVIE_FEATURES_SINK + iteration));
            }
        }
    }

    @Override
    public void close() {
        if (engine != null) AlsFfm.destroyEngine(engine);
    }
}
