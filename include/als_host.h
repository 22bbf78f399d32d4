/*
 * als_host.h -- host-side data layer of libcfk_als.so (C ABI).
 *
 * These are the callers on either side of the hot path, restated natively:
 *   - ingest:   NetflixDataFormatProducer.runProducer      producers/NetflixDataFormatProducer.java:44-60
 *   - blocks:   MRatings2BlocksProcessor / URatings2BlocksProcessor (in-blocks = CSR rows in arrival order)
 *               processors/MRatings2BlocksProcessor.java:48-69, processors/URatings2BlocksProcessor.java:72-92
 *   - sharding: PureModStreamPartitioner.partition = key % numPartitions   producers/PureModStreamPartitioner.java:9-10
 *   - U0:       UFeatureInitializer.process (f[0] = mean rating, f[1..] uniform [0,1))   processors/UFeatureInitializer.java:43-56
 *   - output:   FeatureCollector.calculatePredictionMatrix + EJML MatrixIO.saveDenseCSV   processors/FeatureCollector.java:72-110
 * plus the seeded synthetic Netflix-shape generator used by the benchmark (BASELINE.json configs[2]).
 *
 * Slot layout for G shards (G = 1 for one GPU) and C chunks (default 1): entities of a side are sharded by
 * raw_id % G; inside a shard they are ordered by ascending raw id (rank r = the entity's local row in its
 * shard's block). With S = the largest shard size and Sc = ceil(S / C) slots per shard and chunk,
 *     slot = (r / Sc) * (G * Sc) + shard * Sc + r % Sc            ("chunk-major")
 * so chunk c of the factor matrix (rows [c G Sc, (c+1) G Sc)) holds the G shards' Sc-row pieces back to back,
 * and the exchange of one chunk after it is solved is ONE contiguous all-gather (als_allgather_shard). C = 1
 * gives slot = shard * S + r: the all-gather of equal S-row shards IS the full matrix. For G = 1, slot = rank of
 * the raw id among all ids of that side (= the collector's TreeMap order, FeatureCollector.java:21-22).
 */
#ifndef CFK_ALS_HOST_H
#define CFK_ALS_HOST_H

#include <stdint.h>

#include "als.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct als_dataset als_dataset;

/* Netflix format: "MovieID:" header lines, then "UserID,Rating,Date" lines (date ignored). Lines are
 * parsed exactly as NetflixDataFormatProducer.java:44-60; a malformed line is ALS_ERR_PARSE (the reference
 * producer throws NumberFormatException). Ids must be >= 0 (partition = id % P). */
int als_dataset_load_netflix(const char* path, als_dataset** out);
/* Ratings given in arrival order (movie id, user id, rating) -- e.g. records of movieIds-with-ratings. */
int als_dataset_from_ratings(int64_t n, const int32_t* movie_ids, const int32_t* user_ids, const int16_t* ratings,
                             als_dataset** out);
/* Synthetic Netflix-shape data: user degrees log-normal (median 96, mean ~208, cap 17,653),
 * movie popularity ~ (rank + 320)^-1.85 over a seeded random rank order, ratings drawn from the medium
 * sample's histogram, no duplicate (user, movie) pairs, every entity rated at least once, exactly nnz
 * ratings. Ids are 1..n. Arrival order is movie-major (like the Netflix files). nthreads <= 0: all cores. */
int als_dataset_synthetic_netflix(int64_t n_users, int64_t n_movies, int64_t nnz, uint64_t seed, int nthreads,
                                  als_dataset** out);
/* Synthetic power-law data (BASELINE.json configs[4]: 10M users x 1M items x 2B ratings): user activity
 * log-normal (sigma 1.5, mean nnz / n_users, cap n_items / 10), item popularity ~ rank^-1 over a seeded rank
 * order -- a few items carry millions of ratings (the split-row load-balance stress). Same guarantees as
 * above (exact nnz, no duplicate pairs, every entity rated, ids 1..n, movie-major arrival order). */
int als_dataset_synthetic_powerlaw(int64_t n_users, int64_t n_items, int64_t nnz, uint64_t seed, int nthreads,
                                   als_dataset** out);
/* Shard-restricted forms for the one-process-per-GPU driver: the same dataset, but holding only the ratings of
 * shard `shard` of G = n_shards (movie id % G == shard or user id % G == shard: that rank's in-blocks of both
 * sides, ~2/G of nnz) in the same relative arrival order, plus every user's rating mean for U0. Every shard query
 * for `shard` under G, and als_dataset_init_user_factors, return what the full dataset returns; als_dataset_counts
 * reports all entities but only the kept ratings. Requires every entity rated without the full generator's fix-up
 * pass (true of the configured shapes; ALS_ERR_UNSUPPORTED otherwise). */
int als_dataset_synthetic_powerlaw_shard(int64_t n_users, int64_t n_items, int64_t nnz, uint64_t seed, int nthreads,
                                         int n_shards, int shard, als_dataset** out);
int als_dataset_synthetic_netflix_shard(int64_t n_users, int64_t n_movies, int64_t nnz, uint64_t seed, int nthreads,
                                        int n_shards, int shard, als_dataset** out);
int als_dataset_destroy(als_dataset* ds);

int als_dataset_counts(const als_dataset* ds, int64_t* n_movies, int64_t* n_users, int64_t* nnz);
/* Raw ids of a side in ascending order (n_movies or n_users entries). */
int als_dataset_ids(const als_dataset* ds, int side, int64_t* ids);
/* Arrival-order triples (any pointer may be NULL). */
int als_dataset_ratings(const als_dataset* ds, int32_t* movie_ids, int32_t* user_ids, int16_t* ratings);
/* Number of repeated (user, movie) pairs: the reference's readiness check (MFeatureCalculator.java:65)
 * never fires for such an entity, so the reference hangs; callers reject them (ALS_ERR_DATA). */
int als_dataset_count_duplicates(const als_dataset* ds, int64_t* n_dup);

/* Shard `shard` of `side` under G = n_shards: rows, the shard's first slot (shard * Sc), its entry count, the
 * slots a shard owns (C * Sc, >= its rows) and total slots (G * C * Sc) of this side. */
int als_dataset_shard_info(const als_dataset* ds, int side, int n_shards, int shard, int64_t* n_rows,
                           int64_t* row_offset, int64_t* nnz, int64_t* slots_per_shard, int64_t* n_slots);
/* Chunk count C of `side`'s slot layout (default 1); affects every later slot query of that side (and the
 * opposite side's column indices). */
int als_dataset_set_slot_chunks(als_dataset* ds, int side, int n_chunks);
/* Sc (slots per shard and chunk) and C of `side` under G = n_shards: local row i of a shard's block sits at
 * slot row_offset + (i / Sc) * (G * Sc) + i % Sc (als_set_row_layout(e, side, Sc, G * Sc)). */
int als_dataset_slot_layout(const als_dataset* ds, int side, int n_shards, int64_t* slots_per_chunk, int* n_chunks);
/* The shard's in-block CSR: row_ptr[n_rows+1], col_idx[nnz] = opposite-side SLOTS under the same G,
 * ratings[nnz], row_ids[n_rows] = raw ids (any of col/ratings/row_ids may be NULL). */
int als_dataset_shard_block(const als_dataset* ds, int side, int n_shards, int64_t shard, int64_t* row_ptr,
                            int32_t* col_idx, int16_t* ratings, int64_t* row_ids);
/* The same shard as COO triples in arrival order (rows = local rows, cols = opposite slots): the input of
 * als_set_block_coo, which does the sort into in-blocks on the GPU. Arrays of shard_info's nnz entries. */
int als_dataset_shard_coo(const als_dataset* ds, int side, int n_shards, int64_t shard, int32_t* rows,
                          int32_t* cols, int16_t* ratings);
/* slot_of[i] = slot of the i-th entity of `side` in ascending raw-id order. */
int als_dataset_slots(const als_dataset* ds, int side, int n_shards, int64_t* slot_of);
/* U0 for every user, written at its slot row (out has n_out_rows >= n_slots rows of ld >= k floats;
 * unused slot rows are zeroed). f[0] = (float)mean(ratings) in double (UFeatureInitializer.java:50),
 * f[1..k-1] = u01(seed, raw user id, f): the reference's unseeded Math.random() (UFeatureInitializer.java:55)
 * replaced by a shared counter-based generator (splitmix64; exact floats in [0,1)). */
int als_dataset_init_user_factors(const als_dataset* ds, int num_features, uint64_t seed, int n_shards,
                                  float* out, int64_t ld, int64_t n_out_rows);
float als_u01(uint64_t seed, int64_t raw_id, int32_t feature);

/* FeatureCollector.calculatePredictionMatrix (:90-110): P = U M^T in fp32 (rows: users ascending, columns:
 * movies ascending), widened to double, written in EJML saveDenseCSV layout ("R C real" header, every value
 * followed by one space, one row per line) with Java Double.toString-style shortest round-trip values. */
int als_write_prediction_csv(const char* path, const float* U, int64_t n_users, int64_t ldu, const float* M,
                             int64_t n_movies, int64_t ldm, int num_features);
/* The same file from a prediction matrix already computed (e.g. on the GPU by als_predict): P row-major
 * n_users x n_movies. */
int als_write_prediction_matrix_csv(const char* path, const float* P, int64_t n_users, int64_t n_movies);

/* ---- Kafka wire formats (big-endian, as the reference's serializers write them) ----
 * FeatureMessage = i32 id | i32 n_deps | n_deps x i32 dependent id | i32 num_features | num_features x f32
 *   (FeatureMessageSerializer.java:27-37, ListSerializer.java:72-84, FloatArraySerializer.java:15-24;
 *   NaN written as Float.floatToIntBits' canonical 0x7fc00000). Size = 12 + 4 n_deps + 4 num_features. */
int64_t als_feature_message_size(int64_t n_deps, int num_features);
/* *length = the message size (also when the buffer is too small). */
int als_feature_message_encode(int32_t id, const int32_t* deps, int64_t n_deps, const float* features,
                               int num_features, uint8_t* out, int64_t capacity, int64_t* length);
/* FeatureMessageDeserializer.java:30-56: the dependent-id count is inferred from `length` and num_features
 * (= ALSApp.NUM_FEATURES); inconsistent lengths or counts are ALS_ERR_PARSE. deps may be NULL (count only). */
int als_feature_message_decode(const uint8_t* data, int64_t length, int num_features, int32_t* id, int32_t* deps,
                               int64_t deps_capacity, int64_t* n_deps, float* features);
/* IdRatingPairMessage = i32 id | i16 rating, 6 bytes (IdRatingPairMessageSerializer.java:24-33). */
int als_id_rating_encode(int32_t id, int16_t rating, uint8_t* out6);
int als_id_rating_decode(const uint8_t* data, int64_t length, int32_t* id, int16_t* rating);
/* The out-block fan-out of one half (MFeatureCalculator.java:122-131, UFeatureCalculator.java:124-128,
 * UFeatureInitializer.java:61-64): for every entity of `side` in ascending raw id, one FeatureMessage per
 * partition of its out-block (partitions in first-appearance order over its in-block), carrying the in-block
 * ids with id % n_partitions == partition in arrival order; keys[m] = that partition (the record key).
 * factors: row i = the i-th entity in ascending raw-id order, stride ld floats. out == NULL: size query
 * (*length bytes, *n_messages messages). offsets[m] = byte offset of message m in out. */
int als_encode_feature_messages(const als_dataset* ds, int side, int n_partitions, int num_features,
                                const float* factors, int64_t ld, uint8_t* out, int64_t capacity, int64_t* length,
                                int64_t* n_messages, int32_t* keys, int64_t* offsets, int64_t messages_capacity);

#ifdef __cplusplus
}
#endif
#endif /* CFK_ALS_HOST_H */
