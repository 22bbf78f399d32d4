package de.hpi.collaborativefilteringkafka.processors;

import de.hpi.collaborativefilteringkafka.apps.ALSApp;
import de.hpi.collaborativefilteringkafka.messages.FeatureMessage;
import de.hpi.collaborativefilteringkafka.nativeals.AlsNative;
import org.apache.kafka.streams.processor.AbstractProcessor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.PunctuationType;

import java.sql.Timestamp;
import java.time.Duration;
import java.util.TreeMap;

/**
 * Drop-in replacement of processors/FeatureCollector.java. Collection, the 1 s stability punctuator and the file
 * name are unchanged (:41-69, :103-106); calculatePredictionMatrix (:90-110) runs on the GPU instead of EJML:
 * the final factors go to one engine in ascending-id order (the TreeMaps' order, :72-88), als_predict computes
 * U M^T as Java-float dots (EJML multTransB's sequential float dot, so the reference's digits), and
 * als_write_prediction_matrix_csv writes EJML's saveDenseCSV layout of the double-widened values.
 */
public class NativeFeatureCollector extends AbstractProcessor<Integer, FeatureMessage> {
    private ProcessorContext context;
    private final TreeMap<Integer, float[]> mFeaturesMap = new TreeMap<>();
    private final TreeMap<Integer, float[]> uFeaturesMap = new TreeMap<>();
    private int mostRecentMFeaturesMapSize;
    private int mostRecentUFeaturesMapSize;
    private boolean hasPredictionMatrixBeenComputed;

    @Override
    public void init(final ProcessorContext context) {
        this.context = context;
        this.context.schedule(Duration.ofSeconds(1), PunctuationType.WALL_CLOCK_TIME, timestamp -> {
            if (mFeaturesMap.size() == ALSApp.NUM_MOVIES && uFeaturesMap.size() == ALSApp.NUM_USERS
                    && !hasPredictionMatrixBeenComputed) {
                if (mFeaturesMap.size() == mostRecentMFeaturesMapSize && uFeaturesMap.size() == mostRecentUFeaturesMapSize) {
                    System.out.println(String.format("Start Prediction Matrix Computation at %s",
                            new Timestamp(System.currentTimeMillis())));
                    calculatePredictionMatrix();
                    hasPredictionMatrixBeenComputed = true;
                } else {
                    mostRecentMFeaturesMapSize = mFeaturesMap.size();
                    mostRecentUFeaturesMapSize = uFeaturesMap.size();
                }
            }
        });
    }

    @Override
    public void process(final Integer partition, final FeatureMessage msg) {
        if (context.topic().equals(ALSApp.MOVIE_FEATURES_TOPIC + "-" + ALSApp.NUM_ALS_ITERATIONS)) {
            mFeaturesMap.put(msg.id, msg.features);
        } else if (context.topic().equals(ALSApp.USER_FEATURES_TOPIC + "-" + ALSApp.NUM_ALS_ITERATIONS)) {
            uFeaturesMap.put(msg.id, msg.features);
        }
    }

    /** The features of a TreeMap, row i = the i-th smallest id, as one row-major float matrix. */
    private static float[] flatten(TreeMap<Integer, float[]> rows) {
        final int k = ALSApp.NUM_FEATURES;
        final float[] out = new float[rows.size() * k];
        int i = 0;
        for (float[] f : rows.values()) System.arraycopy(f, 0, out, k * i++, k);
        return out;
    }

    private void calculatePredictionMatrix() {
        final int k = ALSApp.NUM_FEATURES, nu = uFeaturesMap.size(), nm = mFeaturesMap.size();
        final long engine = AlsNative.create(0, k, AlsNative.F32);
        try {
            AlsNative.allocFactors(engine, AlsNative.SIDE_USER, nu);
            AlsNative.allocFactors(engine, AlsNative.SIDE_MOVIE, nm);
            AlsNative.writeFactors(engine, AlsNative.SIDE_USER, 0, flatten(uFeaturesMap), k);
            AlsNative.writeFactors(engine, AlsNative.SIDE_MOVIE, 0, flatten(mFeaturesMap), k);
            final long[] urows = new long[nu], mrows = new long[nm];
            for (int i = 0; i < nu; i++) urows[i] = i;
            for (int j = 0; j < nm; j++) mrows[j] = j;
            final float[] prediction = new float[nu * nm];
            AlsNative.predict(engine, urows, mrows, prediction);
            System.out.println(String.format("Done at %s", new Timestamp(System.currentTimeMillis())));
            AlsNative.writePredictionMatrixCsv("./predictions/prediction_matrix_" + new Timestamp(System.currentTimeMillis()),
                    prediction, nu, nm);
        } finally {
            AlsNative.destroy(engine);
        }
    }

    @Override
    public void close() {}
}
