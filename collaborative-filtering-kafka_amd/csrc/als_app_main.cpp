// als_app -- command-line replacement for ALSAppRunner (apps/ALSAppRunner.java:10-37) on 1..G MI355X.
//
//   als_app NUM_PARTITIONS NUM_FEATURES LAMBDA NUM_ITERATIONS dataset NUM_MOVIES NUM_USERS
//           [--precision f32|f64] [--seed S] [--gpus G] [--out DIR]
//
// Same 7 positional arguments (README.md:35); the extras are optional trailing flags. The run follows the
// reference topology (ALSApp.java:52-184) bulk-synchronously: ingest (NetflixDataFormatProducer), in-blocks
// (M/URatings2BlocksProcessor), U0 after the EOF barrier (UFeatureInitializer), N iterations of
// MFeatureCalculator-i then UFeatureCalculator-i on the GPUs, and FeatureCollector's prediction matrix written
// to ./predictions/prediction_matrix_<timestamp> in EJML dense-CSV layout.
// NUM_PARTITIONS drives the sharding: G = the largest divisor of NUM_PARTITIONS that is <= the number of GPUs
// (or --gpus), so that shard(id) = id % G = (id % NUM_PARTITIONS) % G (PureModStreamPartitioner.java:9-10).
// One process drives the G engines (one per GPU); every half ends with an RCCL all-gather of each shard
// (als_allgather_shard), the replacement for the per-iteration feature topics (ALSApp.java:105-151).
// Deviations that turn reference hangs into errors: duplicate (user, movie) pairs, and NUM_MOVIES /
// NUM_USERS not equal to the rated-entity counts (FeatureCollector.java:43 would never fire).
#include <sys/stat.h>
#include <sys/time.h>

#include <cerrno>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <ctime>
#include <algorithm>
#include <string>
#include <vector>

#include "als.h"
#include "als_host.h"

namespace {

// java.sql.Timestamp.toString() of System.currentTimeMillis(): "yyyy-mm-dd hh:mm:ss.f" (fraction without
// trailing zeros, at least one digit).
std::string java_timestamp() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    struct tm lt;
    time_t sec = tv.tv_sec;
    localtime_r(&sec, &lt);
    char buf[64];
    strftime(buf, sizeof(buf), "%Y-%m-%d %H:%M:%S", &lt);
    char frac[16];
    snprintf(frac, sizeof(frac), "%03d", (int)(tv.tv_usec / 1000));
    std::string f(frac);
    while (f.size() > 1 && f.back() == '0') f.pop_back();
    return std::string(buf) + "." + f;
}

bool parse_int(const char* s, long long lo, long long hi, long long& out) {
    char* end = nullptr;
    errno = 0;
    long long v = strtoll(s, &end, 10);
    if (errno || !end || *end || end == s || v < lo || v > hi) return false;
    out = v;
    return true;
}

int die(const char* what) {
    fprintf(stderr, "als_app: %s: %s\n", what, als_last_error());
    return 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc - 1 < 7) {   // ALSAppRunner.java:11-14
        printf("\x1b[31mARGUMENTS MISSING\x1b[0m\n");
        return 0;
    }
    long long P, K, N, NM, NU;
    if (!parse_int(argv[1], 1, INT_MAX, P) || !parse_int(argv[2], 1, 1024, K) || !parse_int(argv[4], 0, INT_MAX, N) ||
        !parse_int(argv[6], 0, INT_MAX, NM) || !parse_int(argv[7], 0, INT_MAX, NU)) {
        fprintf(stderr, "als_app: bad integer argument (NUM_FEATURES must be 1..1024)\n");
        return 1;
    }
    char* end = nullptr;
    const float lambda = strtof(argv[3], &end);   // Float.parseFloat (ALSAppRunner.java:19)
    if (!end || *end) {
        fprintf(stderr, "als_app: bad LAMBDA\n");
        return 1;
    }
    const char* dataset = argv[5];
    int precision = ALS_F32;
    unsigned long long seed = 42;
    int gpus = 0;
    std::string outdir = "./predictions";
    for (int i = 8; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--precision" && i + 1 < argc) {
            std::string p = argv[++i];
            if (p == "f64") precision = ALS_F64;
            else if (p == "f32") precision = ALS_F32;
            else { fprintf(stderr, "als_app: --precision f32|f64\n"); return 1; }
        } else if (a == "--seed" && i + 1 < argc) {
            seed = strtoull(argv[++i], nullptr, 10);
        } else if (a == "--gpus" && i + 1 < argc) {
            gpus = atoi(argv[++i]);
        } else if (a == "--out" && i + 1 < argc) {
            outdir = argv[++i];
        } else {
            fprintf(stderr, "als_app: unknown option %s\n", a.c_str());
            return 1;
        }
    }
    int ndev = 0;
    if (als_device_count(&ndev) != ALS_OK || ndev < 1) return die("no GPU");
    const int cap = gpus > 0 ? std::min(gpus, ndev) : ndev;
    int G = 1;
    for (int g = 1; g <= cap; ++g)
        if (P % g == 0) G = g;

    printf("Start at %s\n", java_timestamp().c_str());
    als_dataset* ds = nullptr;
    if (als_dataset_load_netflix(dataset, &ds) != ALS_OK) return die("ingest");
    printf("Producer is done at %s\n", java_timestamp().c_str());
    int64_t nm, nu, nnz, dups = 0;
    als_dataset_counts(ds, &nm, &nu, &nnz);
    if (als_dataset_count_duplicates(ds, &dups) != ALS_OK) return die("duplicates");
    if (dups > 0) {
        fprintf(stderr, "als_app: %lld duplicate (user, movie) pairs: the reference topology never completes on such "
                        "input (MFeatureCalculator.java:65)\n", (long long)dups);
        return 1;
    }
    if (nm != NM || nu != NU) {
        fprintf(stderr, "als_app: NUM_MOVIES/NUM_USERS = %lld/%lld but the dataset rates %lld movies and %lld users; "
                        "the reference collector would wait forever (FeatureCollector.java:43)\n",
                (long long)NM, (long long)NU, (long long)nm, (long long)nu);
        return 1;
    }
    printf("Got EOF: %lld ratings, %lld movies, %lld users (NUM_PARTITIONS=%lld -> %d GPU shard%s)\n", (long long)nnz,
           (long long)nm, (long long)nu, P, G, G > 1 ? "s" : "");

    // One engine per GPU: shard g's in-blocks of both sides + full replicas of both factor matrices (slot order).
    const int k = (int)K;
    std::vector<als_engine*> eng(G, nullptr);
    int64_t S[2] = {0, 0}, n_slots[2] = {0, 0};
    for (int g = 0; g < G; ++g) {
        if (als_engine_create(g, k, precision, &eng[g]) != ALS_OK) return die("engine");
        for (int side = 0; side < 2; ++side) {
            int64_t n_rows, row_off, bnnz, o_rows, o_off, o_nnz, o_S;
            als_dataset_shard_info(ds, side, G, g, &n_rows, &row_off, &bnnz, &S[side], &n_slots[side]);
            als_dataset_shard_info(ds, 1 - side, G, g, &o_rows, &o_off, &o_nnz, &o_S, &n_slots[1 - side]);
            std::vector<int64_t> rp(n_rows + 1);
            std::vector<int32_t> col(bnnz);
            std::vector<int16_t> rat(bnnz);
            if (als_dataset_shard_block(ds, side, G, g, rp.data(), col.data(), rat.data(), nullptr) != ALS_OK)
                return die("blocks");
            if (als_set_block(eng[g], side, n_rows, row_off, n_slots[1 - side], rp.data(), col.data(), rat.data()) !=
                ALS_OK)
                return die("set_block");
            if (als_alloc_factors(eng[g], side, n_slots[side]) != ALS_OK) return die("alloc");
        }
    }
    // the communicator is created for G = 1 too, so a one-GPU run takes the same exchange path
    if (als_comm_init_group(eng.data(), G) != ALS_OK) return die("RCCL communicator");
    const int64_t nu_slots = n_slots[ALS_SIDE_USER];
    std::vector<float> U0((size_t)nu_slots * k);
    if (als_dataset_init_user_factors(ds, k, seed, G, U0.data(), k, nu_slots) != ALS_OK) return die("init");
    std::vector<double> U0d;
    if (precision == ALS_F64) U0d.assign(U0.begin(), U0.end());
    for (int g = 0; g < G; ++g) {
        const void* src = precision == ALS_F32 ? (const void*)U0.data() : (const void*)U0d.data();
        if (als_write_factors(eng[g], ALS_SIDE_USER, 0, nu_slots, src, k) != ALS_OK) return die("upload");
    }
    // One half = every engine's solve (asynchronous, one GPU each), then the grouped all-gather of every shard
    // (MFeatureCalculator / UFeatureCalculator fan-out, MFeatureCalculator.java:106-132).
    auto half = [&](int side) -> bool {
        for (int g = 0; g < G; ++g)
            if (als_solve_half(eng[g], side, lambda) != ALS_OK) return false;
        if (als_comm_group_start() != ALS_OK) return false;
        for (int g = 0; g < G; ++g)
            if (als_allgather_shard(eng[g], side, S[side], 0) != ALS_OK) return false;   // one chunk
        return als_comm_group_end() == ALS_OK;
    };
    struct timeval t0, t1;
    gettimeofday(&t0, nullptr);
    for (long long it = 0; it < N; ++it) {
        if (!half(ALS_SIDE_MOVIE)) return die("movie half");
        if (!half(ALS_SIDE_USER)) return die("user half");
    }
    for (int g = 0; g < G; ++g)
        if (als_synchronize(eng[g]) != ALS_OK) return die("sync");
    gettimeofday(&t1, nullptr);
    const double secs = (t1.tv_sec - t0.tv_sec) + 1e-6 * (t1.tv_usec - t0.tv_usec);
    double se = 0;
    int64_t cnt = 0;
    for (int g = 0; g < G; ++g) {
        double s1 = 0;
        int64_t c1 = 0;
        if (als_sq_error(eng[g], ALS_SIDE_MOVIE, &s1, &c1) != ALS_OK) return die("sq_error");
        se += s1;
        cnt += c1;
    }
    printf("ALS: %lld iterations in %.3f s (%.3e ratings/s per iteration); MSE %.6f RMSE %.6f\n", N, secs,
           N > 0 ? (double)nnz * N / secs : 0.0, cnt ? se / cnt : 0.0, cnt ? std::sqrt(se / cnt) : 0.0);

    // FeatureCollector: factors in ascending id order (their slots in engine 0's gathered replicas); U M^T on the
    // GPU with the collector's Java-float dot, then the EJML CSV text on the host.
    printf("Start Prediction Matrix Computation at %s\n", java_timestamp().c_str());
    std::vector<int64_t> urows(nu), mrows(nm);
    if (als_dataset_slots(ds, ALS_SIDE_USER, G, urows.data()) != ALS_OK ||
        als_dataset_slots(ds, ALS_SIDE_MOVIE, G, mrows.data()) != ALS_OK)
        return die("slots");
    std::vector<float> pred((size_t)nu * (size_t)nm);
    if (als_predict(eng[0], urows.data(), nu, mrows.data(), nm, pred.data()) != ALS_OK) return die("predict");
    mkdir(outdir.c_str(), 0755);
    const std::string path = outdir + "/prediction_matrix_" + java_timestamp();
    printf("Done at %s\n", java_timestamp().c_str());
    if (als_write_prediction_matrix_csv(path.c_str(), pred.data(), nu, nm) != ALS_OK) return die("csv");
    printf("Prediction matrix: %s\n", path.c_str());
    for (auto* e : eng) als_engine_destroy(e);
    als_dataset_destroy(ds);
    return 0;
}
