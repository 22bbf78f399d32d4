package de.hpi.collaborativefilteringkafka.apps;

import de.hpi.collaborativefilteringkafka.processors.MRatings2BlocksProcessor;
import de.hpi.collaborativefilteringkafka.processors.NativeFeatureCollector;
import de.hpi.collaborativefilteringkafka.processors.NativeMFeatureCalculator;
import de.hpi.collaborativefilteringkafka.processors.NativeUFeatureCalculator;
import de.hpi.collaborativefilteringkafka.processors.UFeatureInitializer;
import de.hpi.collaborativefilteringkafka.processors.URatings2BlocksProcessor;
import de.hpi.collaborativefilteringkafka.producers.PureModStreamPartitioner;
import de.hpi.collaborativefilteringkafka.serdes.FeatureMessage.FeatureMessageDeserializer;
import de.hpi.collaborativefilteringkafka.serdes.FeatureMessage.FeatureMessageSerializer;
import de.hpi.collaborativefilteringkafka.serdes.List.ListSerde;
import org.apache.kafka.common.serialization.Serde;
import org.apache.kafka.common.serialization.Serdes;
import org.apache.kafka.streams.Topology;
import org.apache.kafka.streams.state.StoreBuilder;
import org.apache.kafka.streams.state.Stores;

import java.util.ArrayList;
import java.util.Properties;

/**
 * ALSApp with the GPU hot path: the topology of apps/ALSApp.java:52-184 -- same topics, store names, sources,
 * sinks, partitioner and node names, so the CLI (ALSAppRunner.java:11-23), setup.sh's topics and the collector's
 * CSV stay as they are -- with the per-iteration calculators and the collector swapped for their native
 * counterparts (NativeMFeatureCalculator / NativeUFeatureCalculator, NativeFeatureCollector). Block builders,
 * the EOF barrier and the U0 initialiser are the reference's own processors. ALSAppRunner switches by
 * constructing NativeALSApp instead of ALSApp (same constructor).
 */
public class NativeALSApp extends ALSApp {
    public NativeALSApp(int numPartitions, int numFeatures, float alsLambda, int numAlsIterations, int numMovies,
                        int numUsers) {
        super(numPartitions, numFeatures, alsLambda, numAlsIterations, numMovies, numUsers);
    }

    /** In-memory key-value store, changelog disabled (ALSApp.java:53-83). */
    @SuppressWarnings({"rawtypes", "unchecked"})
    private static StoreBuilder store(String name, Serde<?> element) {
        return Stores.keyValueStoreBuilder(Stores.inMemoryKeyValueStore(name), Serdes.Integer(),
                new ListSerde(ArrayList.class, element)).withLoggingDisabled();
    }

    /** A FeatureMessage sink partitioned by key % P (PureModStreamPartitioner.java:9-10). */
    private static void featureSink(Topology t, String name, String topic, String parent) {
        t.addSink(name, topic, Serdes.Integer().serializer(), new FeatureMessageSerializer(),
                new PureModStreamPartitioner<Integer, Object>(), parent);
    }

    private static void featureSource(Topology t, String name, String topic) {
        t.addSource(name, Serdes.Integer().deserializer(), new FeatureMessageDeserializer(), topic);
    }

    @Override
    public Topology getTopology(Properties properties) {
        final Topology t = new Topology();
        // block builders + EOF barrier + U0 (ALSApp.java:85-113): unchanged reference processors
        t.addSource("movieids-with-ratings-source", MOVIEIDS_WITH_RATINGS_TOPIC)
         .addProcessor("MRatings2Blocks", MRatings2BlocksProcessor::new, "movieids-with-ratings-source")
         .addStateStore(store(M_INBLOCKS_UID_STORE, Serdes.Integer()), "MRatings2Blocks")
         .addStateStore(store(M_INBLOCKS_RATINGS_STORE, Serdes.Short()), "MRatings2Blocks")
         .addStateStore(store(M_OUTBLOCKS_STORE, Serdes.Short()), "MRatings2Blocks")
         .addSink("userids-to-movieids-ratings-sink", USERIDS_TO_MOVIEIDS_RATINGS_TOPIC,
                  new PureModStreamPartitioner<Integer, Object>(), "MRatings2Blocks")
         .addSource("userids-to-movieids-ratings-source", USERIDS_TO_MOVIEIDS_RATINGS_TOPIC)
         .addProcessor("URatings2Blocks", URatings2BlocksProcessor::new, "userids-to-movieids-ratings-source")
         .addStateStore(store(U_INBLOCKS_MID_STORE, Serdes.Integer()), "URatings2Blocks")
         .addStateStore(store(U_INBLOCKS_RATINGS_STORE, Serdes.Short()), "URatings2Blocks")
         .addStateStore(store(U_OUTBLOCKS_STORE, Serdes.Short()), "URatings2Blocks")
         .addSink("eof-sink", EOF_TOPIC, new PureModStreamPartitioner<Integer, Object>(), "URatings2Blocks")
         .addSource("eof-source", EOF_TOPIC)
         .addProcessor("UFeatureInitializer", UFeatureInitializer::new, "eof-source")
         .connectProcessorAndStateStores("UFeatureInitializer", U_INBLOCKS_MID_STORE, U_INBLOCKS_RATINGS_STORE,
                                         U_OUTBLOCKS_STORE);
        featureSink(t, USER_FEATURES_SINK + 0, USER_FEATURES_TOPIC + "-0", "UFeatureInitializer");

        // the unrolled ALS loop (ALSApp.java:115-151): per iteration one native movie and one native user calculator
        // on the shared in-block stores; the task's instances share one GPU engine per side (TaskEngine)
        for (int i = 0; i < NUM_ALS_ITERATIONS; i++) {
            final String m = "MFeatureCalculator-" + i, u = "UFeatureCalculator-" + i;
            featureSource(t, "user-features-source-" + i, USER_FEATURES_TOPIC + "-" + i);
            t.addProcessor(m, NativeMFeatureCalculator::new, "user-features-source-" + i);
            featureSink(t, MOVIE_FEATURES_SINK + i, MOVIE_FEATURES_TOPIC + "-" + i, m);
            t.connectProcessorAndStateStores(m, M_INBLOCKS_UID_STORE, M_INBLOCKS_RATINGS_STORE, M_OUTBLOCKS_STORE);
            featureSource(t, "movie-features-source-" + i, MOVIE_FEATURES_TOPIC + "-" + i);
            t.addProcessor(u, NativeUFeatureCalculator::new, "movie-features-source-" + i);
            // user-features-N has one partition (setup.sh:23-24): the collector's input
            featureSink(t, USER_FEATURES_SINK + (i + 1), USER_FEATURES_TOPIC + "-" + (i + 1), u);
            t.connectProcessorAndStateStores(u, U_INBLOCKS_MID_STORE, U_INBLOCKS_RATINGS_STORE, U_OUTBLOCKS_STORE);
        }
        // final movie factors M_{N-1} (MFeatureCalculator.java:117-123) and the collector (ALSApp.java:153-181)
        featureSink(t, MOVIE_FEATURES_SINK + NUM_ALS_ITERATIONS, MOVIE_FEATURES_TOPIC + "-" + NUM_ALS_ITERATIONS,
                    "MFeatureCalculator-" + (NUM_ALS_ITERATIONS - 1));
        featureSource(t, "movie-features-final-source", MOVIE_FEATURES_TOPIC + "-" + NUM_ALS_ITERATIONS);
        featureSource(t, "user-features-final-source", USER_FEATURES_TOPIC + "-" + NUM_ALS_ITERATIONS);
        t.addProcessor("FeatureCollector", NativeFeatureCollector::new, "user-features-final-source",
                       "movie-features-final-source");
        return t;
    }
}
