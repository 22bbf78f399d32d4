package de.hpi.collaborativefilteringkafka.processors;

import de.hpi.collaborativefilteringkafka.apps.ALSApp;
import de.hpi.collaborativefilteringkafka.messages.FeatureMessage;
import de.hpi.collaborativefilteringkafka.nativeals.AlsNative;
import de.hpi.collaborativefilteringkafka.nativeals.TaskEngine;
import org.apache.kafka.streams.processor.AbstractProcessor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.To;
import org.apache.kafka.streams.state.KeyValueStore;

import java.util.ArrayList;
import java.util.stream.Collectors;

/**
 * Drop-in replacement of processors/MFeatureCalculator.java: same stores, same input records (user-features-i),
 * same output records and sinks (:106-132), but the partition's whole movie half is ONE GPU call
 * (TaskEngine.solve -> als_solve_half) instead of one EJML solve per movie (:66-104). The task's N instances
 * (MFeatureCalculator-0..N-1, ALSApp.java:115-132) share one engine (TaskEngine.acquire).
 */
public class NativeMFeatureCalculator extends AbstractProcessor<Integer, FeatureMessage> {
    private ProcessorContext context;
    private KeyValueStore<Integer, ArrayList<Integer>> mInBlocksUidStore;
    private KeyValueStore<Integer, ArrayList<Short>> mInBlocksRatingsStore;
    private KeyValueStore<Integer, ArrayList<Short>> mOutBlocksStore;
    private TaskEngine engine;

    @Override
    @SuppressWarnings("unchecked")
    public void init(final ProcessorContext context) {
        this.context = context;
        this.mInBlocksUidStore = (KeyValueStore<Integer, ArrayList<Integer>>) context.getStateStore(ALSApp.M_INBLOCKS_UID_STORE);
        this.mInBlocksRatingsStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.M_INBLOCKS_RATINGS_STORE);
        this.mOutBlocksStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.M_OUTBLOCKS_STORE);
        this.engine = TaskEngine.acquire(context.taskId(), AlsNative.SIDE_MOVIE);
    }

    @Override
    public void process(final Integer partition, final FeatureMessage msg) {
        engine.ensureBlocks(mInBlocksUidStore, mInBlocksRatingsStore);   // after the EOF barrier: stores complete
        final String sourceTopic = context.topic();
        final int iteration = Integer.parseInt(sourceTopic.substring(sourceTopic.length() - 1));   // as :106-107
        if (!engine.stage(iteration, msg.id, msg.features)) return;   // readiness of the whole half (:65)

        final float[] solved = engine.solve(iteration, ALSApp.ALS_LAMBDA);
        final int[] movieIds = engine.rowIds();
        for (int r = 0; r < movieIds.length; r++) {     // unchanged fan-out, MFeatureCalculator.java:106-132
            final int movieId = movieIds[r];
            final ArrayList<Integer> dependentUids = mInBlocksUidStore.get(movieId);
            final FeatureMessage out = new FeatureMessage(movieId, dependentUids, TaskEngine.row(solved, r));
            if (iteration == ALSApp.NUM_ALS_ITERATIONS - 1) {
                context.forward(0, out, To.child(ALSApp.MOVIE_FEATURES_SINK + ALSApp.NUM_ALS_ITERATIONS));
            }
            for (int targetPartition : mOutBlocksStore.get(movieId)) {
                out.setDependentIds(dependentUids.stream()
                        .filter(id -> (id % ALSApp.NUM_PARTITIONS) == targetPartition)
                        .collect(Collectors.toCollection(ArrayList::new)));
                context.forward(targetPartition, out, To.child(ALSApp.MOVIE_FEATURES_SINK + iteration));
            }
        }
    }

    @Override
    public void close() {
        if (engine != null) engine.release();
    }
}
