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
 * Drop-in replacement of processors/UFeatureCalculator.java: same stores (u-inblocks-mid, u-inblocks-ratings,
 * u-outblocks), same input records (movie-features-i) and the same output rule (:106-132): iteration i writes to
 * user-features-(i+1); on the last iteration ONLY to the collector's single-partition topic, with the full
 * dependent list (:117-123), otherwise one record per out-block partition with the dependent movie ids filtered
 * by id % NUM_PARTITIONS (:124-131). The partition's whole user half is ONE GPU call (TaskEngine.solve ->
 * als_solve_half) instead of one EJML solve per user (:66-104); the N instances of the task share one engine.
 */
public class NativeUFeatureCalculator extends AbstractProcessor<Integer, FeatureMessage> {
    private ProcessorContext context;
    private KeyValueStore<Integer, ArrayList<Integer>> uInBlocksMidStore;
    private KeyValueStore<Integer, ArrayList<Short>> uInBlocksRatingsStore;
    private KeyValueStore<Integer, ArrayList<Short>> uOutBlocksStore;
    private TaskEngine engine;

    @Override
    @SuppressWarnings("unchecked")
    public void init(final ProcessorContext context) {
        this.context = context;
        this.uInBlocksMidStore = (KeyValueStore<Integer, ArrayList<Integer>>) context.getStateStore(ALSApp.U_INBLOCKS_MID_STORE);
        this.uInBlocksRatingsStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.U_INBLOCKS_RATINGS_STORE);
        this.uOutBlocksStore = (KeyValueStore<Integer, ArrayList<Short>>) context.getStateStore(ALSApp.U_OUTBLOCKS_STORE);
        this.engine = TaskEngine.acquire(context.taskId(), AlsNative.SIDE_USER);
    }

    @Override
    public void process(final Integer partition, final FeatureMessage msg) {
        engine.ensureBlocks(uInBlocksMidStore, uInBlocksRatingsStore);
        final String sourceTopic = context.topic();
        final int sourceTopicIteration = Integer.parseInt(sourceTopic.substring(sourceTopic.length() - 1));   // :106-107
        final int sinkTopicIteration = sourceTopicIteration + 1;
        if (!engine.stage(sourceTopicIteration, msg.id, msg.features)) return;

        final float[] solved = engine.solve(sourceTopicIteration, ALSApp.ALS_LAMBDA);
        final int[] userIds = engine.rowIds();
        for (int r = 0; r < userIds.length; r++) {
            final int userId = userIds[r];
            final ArrayList<Integer> dependentMids = uInBlocksMidStore.get(userId);
            final FeatureMessage out = new FeatureMessage(userId, dependentMids, TaskEngine.row(solved, r));
            if (sourceTopicIteration == ALSApp.NUM_ALS_ITERATIONS - 1) {       // last iteration: collector only
                context.forward(0, out, To.child(ALSApp.USER_FEATURES_SINK + sinkTopicIteration));
            } else {
                for (int targetPartition : uOutBlocksStore.get(userId)) {
                    out.setDependentIds(dependentMids.stream()
                            .filter(id -> (id % ALSApp.NUM_PARTITIONS) == targetPartition)
                            .collect(Collectors.toCollection(ArrayList::new)));
                    context.forward(targetPartition, out, To.child(ALSApp.USER_FEATURES_SINK + sinkTopicIteration));
                }
            }
        }
    }

    @Override
    public void close() {
        if (engine != null) engine.release();
    }
}
