// als_codec.cpp -- the reference's Kafka wire formats, so the engine can feed or consume
// the real topics: FeatureMessage (serdes/FeatureMessage/FeatureMessageSerializer.java:27-37: writeInt(id),
// ListSerializer<Integer> = writeInt(size) + size x 4-B ints (List/ListSerializer.java:72-84, fixed-length inner),
// FloatArraySerializer = writeInt(length) + writeFloat each (FloatArray/FloatArraySerializer.java:15-24)) and
// IdRatingPairMessage (IdRatingPairMessageSerializer.java:24-33: IntegerSerializer + ShortSerializer), all
// big-endian as java.io.DataOutputStream / Kafka's serializers write them. The decoder mirrors
// FeatureMessageDeserializer.java:30-56, which infers the dependent-id list length from the message length and
// ALSApp.NUM_FEATURES. The out-block fan-out mirrors MFeatureCalculator.java:106-132 / UFeatureCalculator.java:
// 106-132: one message per (entity, partition of its out-block), dependent ids filtered by id % P == partition.
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "als.h"
#include "als_host.h"

namespace cfk_detail {
void set_last_error(const std::string& s);
}

namespace {

int err(int code, const char* msg) {
    cfk_detail::set_last_error(msg);
    return code;
}

inline void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}
inline uint32_t get32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
// DataOutputStream.writeFloat writes Float.floatToIntBits: every NaN becomes the canonical 0x7fc00000
inline uint32_t float_bits(float f) {
    if (f != f) return 0x7fc00000u;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

}  // namespace

extern "C" {

int64_t als_feature_message_size(int64_t n_deps, int num_features) { return 4 + 4 + 4 * n_deps + 4 + 4 * (int64_t)num_features; }

int als_feature_message_encode(int32_t id, const int32_t* deps, int64_t n_deps, const float* features, int num_features,
                               uint8_t* out, int64_t capacity, int64_t* length) {
    if (n_deps < 0 || n_deps > INT32_MAX || num_features < 0 || (n_deps > 0 && !deps) || (num_features > 0 && !features))
        return err(ALS_ERR_INVALID_ARGUMENT, "als_feature_message_encode: bad arguments");
    const int64_t need = als_feature_message_size(n_deps, num_features);
    if (length) *length = need;
    if (!out || capacity < need) return err(ALS_ERR_INVALID_ARGUMENT, "als_feature_message_encode: buffer too small");
    uint8_t* p = out;
    put32(p, (uint32_t)id);
    p += 4;
    put32(p, (uint32_t)n_deps);
    p += 4;
    for (int64_t i = 0; i < n_deps; ++i, p += 4) put32(p, (uint32_t)deps[i]);
    put32(p, (uint32_t)num_features);
    p += 4;
    for (int i = 0; i < num_features; ++i, p += 4) put32(p, float_bits(features[i]));
    return ALS_OK;
}

int als_feature_message_decode(const uint8_t* data, int64_t length, int num_features, int32_t* id, int32_t* deps,
                               int64_t deps_capacity, int64_t* n_deps, float* features) {
    if (!data || num_features < 0) return err(ALS_ERR_INVALID_ARGUMENT, "als_feature_message_decode: bad arguments");
    // FeatureMessageDeserializer.java:33-35: the feature list is 4 * (1 + NUM_FEATURES) bytes at the end
    const int64_t feat_bytes = 4 * (1 + (int64_t)num_features);
    const int64_t dep_bytes = length - 4 - feat_bytes;
    if (dep_bytes < 4) return err(ALS_ERR_PARSE, "FeatureMessage shorter than id + list size + features");
    const int64_t nd = (int32_t)get32(data + 4);
    if (nd < 0 || 4 + 4 * nd != dep_bytes) return err(ALS_ERR_PARSE, "FeatureMessage dependent-id list length mismatch");
    if ((int32_t)get32(data + 4 + dep_bytes) != num_features)
        return err(ALS_ERR_PARSE, "FeatureMessage feature count differs from NUM_FEATURES");
    if (id) *id = (int32_t)get32(data);
    if (n_deps) *n_deps = nd;
    if (deps) {
        if (deps_capacity < nd) return err(ALS_ERR_INVALID_ARGUMENT, "dependent-id buffer too small");
        for (int64_t i = 0; i < nd; ++i) deps[i] = (int32_t)get32(data + 8 + 4 * i);
    }
    if (features) {
        const uint8_t* f = data + 4 + dep_bytes + 4;
        for (int i = 0; i < num_features; ++i) {
            const uint32_t u = get32(f + 4 * i);
            std::memcpy(features + i, &u, 4);
        }
    }
    return ALS_OK;
}

int als_id_rating_encode(int32_t id, int16_t rating, uint8_t* out6) {
    if (!out6) return err(ALS_ERR_INVALID_ARGUMENT, "als_id_rating_encode: out is NULL");
    put32(out6, (uint32_t)id);
    out6[4] = (uint8_t)((uint16_t)rating >> 8);
    out6[5] = (uint8_t)rating;
    return ALS_OK;
}

int als_id_rating_decode(const uint8_t* data, int64_t length, int32_t* id, int16_t* rating) {
    if (!data || length != 6) return err(ALS_ERR_PARSE, "IdRatingPairMessage must be 6 bytes");
    if (id) *id = (int32_t)get32(data);
    if (rating) *rating = (int16_t)(((uint16_t)data[4] << 8) | data[5]);
    return ALS_OK;
}

int als_encode_feature_messages(const als_dataset* ds, int side, int n_partitions, int num_features,
                                const float* factors, int64_t ld, uint8_t* out, int64_t capacity, int64_t* length,
                                int64_t* n_messages, int32_t* keys, int64_t* offsets, int64_t messages_capacity) {
    if (!ds || (side != ALS_SIDE_MOVIE && side != ALS_SIDE_USER) || n_partitions < 1 || n_partitions > INT16_MAX ||
        num_features < 0 || (out && (!factors || ld < num_features)))
        return err(ALS_ERR_INVALID_ARGUMENT, "als_encode_feature_messages: bad arguments");
    int64_t counts[2] = {0, 0}, nnz = 0;
    int rc = als_dataset_counts(ds, &counts[ALS_SIDE_MOVIE], &counts[ALS_SIDE_USER], &nnz);
    if (rc != ALS_OK) return rc;
    const int64_t n_rows = counts[side], n_opp = counts[1 - side];
    // G = 1: one CSR over the whole side, rows in ascending raw id, entries in arrival order (the in-block
    // lists), columns = rank of the opposite raw id
    std::vector<int64_t> row_ptr(n_rows + 1), row_ids(n_rows), opp_ids(n_opp);
    std::vector<int32_t> col(nnz);
    if ((rc = als_dataset_shard_block(ds, side, 1, 0, row_ptr.data(), col.data(), nullptr, row_ids.data())) != ALS_OK)
        return rc;
    if ((rc = als_dataset_ids(ds, 1 - side, opp_ids.data())) != ALS_OK) return rc;

    int64_t total = 0, n_msg = 0;
    std::vector<int32_t> order;          // the out-block: partitions in first-appearance order
    std::vector<int64_t> per_part(n_partitions);
    std::vector<int32_t> deps;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1) {
            if (length) *length = total;
            if (n_messages) *n_messages = n_msg;
            if (!out) return ALS_OK;   // size query
            if (capacity < total) return err(ALS_ERR_INVALID_ARGUMENT, "message buffer too small");
            if ((keys || offsets) && messages_capacity < n_msg)
                return err(ALS_ERR_INVALID_ARGUMENT, "key/offset arrays too small");
            total = 0;
            n_msg = 0;
        }
        for (int64_t r = 0; r < n_rows; ++r) {
            order.clear();
            std::fill(per_part.begin(), per_part.end(), 0);
            for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e) {
                const int32_t p = (int32_t)(opp_ids[col[e]] % n_partitions);
                if (per_part[p]++ == 0) order.push_back(p);
            }
            for (int32_t p : order) {
                const int64_t sz = als_feature_message_size(per_part[p], num_features);
                if (pass == 1) {
                    deps.clear();
                    for (int64_t e = row_ptr[r]; e < row_ptr[r + 1]; ++e)
                        if (opp_ids[col[e]] % n_partitions == p) deps.push_back((int32_t)opp_ids[col[e]]);
                    rc = als_feature_message_encode((int32_t)row_ids[r], deps.data(), (int64_t)deps.size(),
                                                    factors + r * ld, num_features, out + total, capacity - total, nullptr);
                    if (rc != ALS_OK) return rc;
                    if (keys) keys[n_msg] = p;
                    if (offsets) offsets[n_msg] = total;
                }
                total += sz;
                ++n_msg;
            }
        }
    }
    return ALS_OK;
}

}  // extern "C"
