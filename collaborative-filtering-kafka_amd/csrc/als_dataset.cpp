// als_dataset.cpp -- host data layer (include/als_host.h): Netflix-format ingest, in-block (CSR) build,
// id % G sharding into slot order, seeded U0, synthetic Netflix-shape generator, prediction CSV.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include <atomic>
#include <thread>

#include "als_host.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace

// als_last_error() is defined in als_engine.cpp; the data layer keeps its own thread-local message and
// exposes it through the same accessor by forwarding on failure.
extern "C" const char* als_last_error(void);
namespace cfk_detail {
void set_last_error(const std::string& s);
}

struct als_dataset {
    // arrival order (the producer's send order, NetflixDataFormatProducer.java:58)
    std::vector<int32_t> movie, user;
    std::vector<int16_t> rating;
    // derived
    std::vector<int64_t> ids[2];      // ascending raw ids per side (0 = movie, 1 = user)
    std::vector<int32_t> dense[2];    // per rating: dense (ascending-id rank) index of its movie / user
    int chunks[2] = {1, 1};           // chunk-major slot layout per side (als_dataset_set_slot_chunks)
    // a shard-restricted synthetic dataset (als_dataset_synthetic_powerlaw_shard) holds only the ratings of its
    // shard's in-blocks, so U0's rating means come from every user's full rating sum, kept here (per dense user)
    std::vector<int64_t> user_sum, user_cnt;
};

namespace {

int report(int code) {
    if (code != ALS_OK) cfk_detail::set_last_error(g_err);
    return code;
}

void finalize(als_dataset* ds) {
    const int64_t n = (int64_t)ds->rating.size();
    for (int s = 0; s < 2; ++s) {
        const std::vector<int32_t>& raw = s == 0 ? ds->movie : ds->user;
        int32_t mx = 0;
        for (int32_t v : raw) mx = std::max(mx, v);
        // counting presence over [0, max] (ids are bounded by int32 and were checked >= 0)
        std::vector<int32_t> rank((size_t)mx + 1, -1);
        for (int32_t v : raw) rank[v] = 0;
        ds->ids[s].clear();
        for (int64_t v = 0; v <= mx; ++v)
            if (rank[v] == 0) {
                rank[v] = (int32_t)ds->ids[s].size();
                ds->ids[s].push_back(v);
            }
        ds->dense[s].resize(n);
        for (int64_t t = 0; t < n; ++t) ds->dense[s][t] = rank[raw[t]];
    }
}

// Shard geometry of one side under G shards and C chunks (als_host.h "Slot layout"): entity i of shard
// sh = id % G with rank r among that shard's ids (ascending) sits at slot (r / Sc) * (G * Sc) + sh * Sc + r % Sc,
// Sc = ceil(S / C), S = the largest shard. C = 1: slot = sh * S + r (shard-major).
struct ShardMap {
    int G = 1, C = 1;
    int64_t S = 0;                        // rows of the largest shard
    int64_t Sc = 0;                       // slots per shard and chunk
    std::vector<int64_t> slot;            // per dense entity
    std::vector<int32_t> shard;           // per dense entity
    std::vector<int64_t> local;           // per dense entity: its row in its shard's block (= rank)
    std::vector<int64_t> count;           // entities per shard
    int64_t n_slots() const { return (int64_t)C * G * Sc; }
};

ShardMap shard_map(const als_dataset* ds, int side, int G) {
    ShardMap m;
    m.G = G;
    m.C = ds->chunks[side];
    const auto& ids = ds->ids[side];
    m.count.assign(G, 0);
    m.slot.resize(ids.size());
    m.shard.resize(ids.size());
    m.local.resize(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        const int sh = (int)(ids[i] % G);   // PureModStreamPartitioner.java:10
        m.shard[i] = sh;
        m.local[i] = m.count[sh]++;
    }
    m.S = 0;
    for (int64_t c : m.count) m.S = std::max(m.S, c);
    m.Sc = (m.S + m.C - 1) / m.C;
    for (size_t i = 0; i < ids.size(); ++i) {
        const int64_t r = m.local[i];
        m.slot[i] = (r / m.Sc) * ((int64_t)G * m.Sc) + (int64_t)m.shard[i] * m.Sc + r % m.Sc;
    }
    return m;
}

// Java Double.toString layout over the shortest round-trip digits.
std::string java_double(double v) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
    if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
    char buf[64];
    auto res = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
    std::string s(buf, res.ptr);
    std::string sign;
    if (s[0] == '-') {
        sign = "-";
        s = s.substr(1);
    }
    const size_t epos = s.find('e');
    const int exp10 = atoi(s.c_str() + epos + 1);
    std::string digits;
    for (size_t i = 0; i < epos; ++i)
        if (s[i] != '.') digits.push_back(s[i]);
    const double a = std::fabs(v);
    std::string out;
    if (a >= 1e-3 && a < 1e7) {
        if (exp10 >= 0) {
            std::string ip = digits.substr(0, std::min<size_t>(digits.size(), (size_t)exp10 + 1));
            while ((int)ip.size() < exp10 + 1) ip.push_back('0');
            std::string fp = digits.size() > (size_t)exp10 + 1 ? digits.substr(exp10 + 1) : "0";
            out = ip + "." + fp;
        } else {
            out = "0." + std::string((size_t)(-exp10 - 1), '0') + digits;
        }
    } else {
        out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp10);
    }
    return sign + out;
}

uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct Rng {   // xoshiro256** seeded by splitmix64
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        for (auto& w : s) w = seed = mix64(seed);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return (uint64_t)(((__uint128_t)next() * n) >> 64); }
};

}  // namespace

extern "C" {

float als_u01(uint64_t seed, int64_t raw_id, int32_t feature) {
    const uint64_t h = mix64(seed ^ mix64((uint64_t)raw_id * 0x100000001B3ULL + (uint64_t)(uint32_t)feature));
    return (float)(h >> 40) * (1.0f / 16777216.0f);
}

int als_dataset_load_netflix(const char* path, als_dataset** out) {
    if (!path || !out) return report(fail(ALS_ERR_INVALID_ARGUMENT, "NULL argument"));
    *out = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return report(fail(ALS_ERR_IO, "cannot open %s", path));
    std::unique_ptr<als_dataset> ds(new als_dataset());
    // BufferedReader.readLine semantics: a line ends at "\n", "\r" or "\r\n" and may be of any length
    // (NetflixDataFormatProducer.java:44); the file is streamed through a fixed buffer.
    std::vector<char> buf(1 << 20);
    size_t bpos = 0, blen = 0;
    bool eof = false;
    std::string line;
    auto next_line = [&](std::string& out) -> bool {
        out.clear();
        bool any = false;
        for (;;) {
            if (bpos == blen) {
                if (eof) return any;
                blen = fread(buf.data(), 1, buf.size(), f);
                bpos = 0;
                if (blen == 0) {
                    eof = true;
                    return any;
                }
            }
            any = true;
            const char* b = buf.data() + bpos;
            const char* e = buf.data() + blen;
            const char* p = b;
            while (p < e && *p != '\n' && *p != '\r') ++p;
            out.append(b, p);
            bpos += (size_t)(p - b);
            if (p == e) continue;                        // line continues in the next buffer
            const char term = *p;
            ++bpos;
            if (term == '\r') {                          // "\r\n" counts as one terminator
                if (bpos == blen && !eof) {
                    blen = fread(buf.data(), 1, buf.size(), f);
                    bpos = 0;
                    if (blen == 0) eof = true;
                }
                if (bpos < blen && buf[bpos] == '\n') ++bpos;
            }
            return true;
        }
    };
    int64_t current = -1;
    int64_t lineno = 0;
    auto parse_int = [](const char* b, const char* e, int64_t& v) -> bool {
        // Integer.parseInt / Short.parseShort: optional sign, decimal digits only
        if (b == e) return false;
        bool neg = false;
        if (*b == '-' || *b == '+') {
            neg = *b == '-';
            ++b;
            if (b == e) return false;
        }
        int64_t x = 0;
        for (; b < e; ++b) {
            if (*b < '0' || *b > '9') return false;
            x = x * 10 + (*b - '0');
            if (x > (int64_t)1 << 40) return false;
        }
        v = neg ? -x : x;
        return true;
    };
    while (next_line(line)) {
        ++lineno;
        const size_t n = line.size();
        const char* b = line.data();
        const char* e = b + n;
        if (n > 0 && b[n - 1] == ':') {                                   // row.endsWith(":")
            const char* colon = (const char*)memchr(b, ':', n);           // row.split(":")[0]
            int64_t v;
            if (!parse_int(b, colon, v) || v < 0 || v > INT32_MAX) {
                fclose(f);
                return report(fail(ALS_ERR_PARSE, "%s:%lld: bad movie header", path, (long long)lineno));
            }
            current = v;
            continue;
        }
        const char* c1 = (const char*)memchr(b, ',', n);
        const char* c2 = c1 ? (const char*)memchr(c1 + 1, ',', e - c1 - 1) : nullptr;
        const char* rend = c2 ? c2 : e;
        int64_t uid, r;
        if (!c1 || !parse_int(b, c1, uid) || !parse_int(c1 + 1, rend, r) || uid < 0 || uid > INT32_MAX ||
            r < -32768 || r > 32767) {
            fclose(f);
            return report(fail(ALS_ERR_PARSE, "%s:%lld: expected UserID,Rating,Date", path, (long long)lineno));
        }
        if (current < 0) {
            fclose(f);
            return report(fail(ALS_ERR_PARSE, "%s:%lld: rating before the first movie header", path, (long long)lineno));
        }
        ds->movie.push_back((int32_t)current);
        ds->user.push_back((int32_t)uid);
        ds->rating.push_back((int16_t)r);
    }
    fclose(f);
    finalize(ds.get());
    *out = ds.release();
    return ALS_OK;
}

int als_dataset_from_ratings(int64_t n, const int32_t* movie_ids, const int32_t* user_ids, const int16_t* ratings,
                             als_dataset** out) {
    if (!out || n < 0 || (n > 0 && (!movie_ids || !user_ids || !ratings)))
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    *out = nullptr;
    for (int64_t t = 0; t < n; ++t)
        if (movie_ids[t] < 0 || user_ids[t] < 0)
            return report(fail(ALS_ERR_INVALID_ARGUMENT, "negative id at rating %lld", (long long)t));
    std::unique_ptr<als_dataset> ds(new als_dataset());
    ds->movie.assign(movie_ids, movie_ids + n);
    ds->user.assign(user_ids, user_ids + n);
    ds->rating.assign(ratings, ratings + n);
    finalize(ds.get());
    *out = ds.release();
    return ALS_OK;
}

}  // extern "C"

namespace {

// Shape of a synthetic rating matrix: log-normal user activity (mu, sigma of the log, per-user cap; scaled to
// exactly nnz) and item popularity w(rank) over a seeded random rank order.
struct SynthSpec {
    double mu, sigma;
    int64_t cap;
    double rank_offset, exponent;     // w(rank) = (rank + 1 + rank_offset)^-exponent
    uint64_t perm_salt;
};

// G > 1: keep only the ratings of shard `keep` (movie id % G == keep or user id % G == keep: the in-blocks of both
// sides of that shard) -- the same ratings, in the same relative arrival order, as the full dataset's (G = 1).
int synthesize(const SynthSpec& sp, int64_t n_users, int64_t n_movies, int64_t nnz, uint64_t seed, int nthreads,
               als_dataset** out, int G = 1, int keep = 0) {
    if (!out) return report(fail(ALS_ERR_INVALID_ARGUMENT, "out is NULL"));
    *out = nullptr;
    if (G < 1 || keep < 0 || keep >= G) return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad shard %d of %d", keep, G));
    if (n_users < 1 || n_movies < 1 || n_users > INT32_MAX - 1 || n_movies > INT32_MAX - 1)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad entity counts"));
    if (nnz < std::max(n_users, n_movies) || nnz > n_users * n_movies / 2)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "nnz must be in [max(n_users, n_movies), n_users*n_movies/2]"));
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    nthreads = std::min(nthreads, 64);
    const double mu = sp.mu, sigma = sp.sigma;
    const int64_t cap = std::min<int64_t>(sp.cap, n_movies);
    if (cap * n_users < nnz) return report(fail(ALS_ERR_INVALID_ARGUMENT, "nnz exceeds n_users * per-user cap"));
    std::vector<int64_t> deg(n_users);
    {
        Rng rng(mix64(seed ^ 0xDE6DE6ULL));
        std::vector<double> raw(n_users);
        double sum = 0;
        for (int64_t u = 0; u < n_users; ++u) {
            // Box-Muller
            double u1 = rng.uniform(), u2 = rng.uniform();
            if (u1 < 1e-300) u1 = 1e-300;
            const double z = std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
            raw[u] = std::exp(mu + sigma * z);
            sum += raw[u];
        }
        const double scale = (double)nnz / sum;
        int64_t tot = 0;
        for (int64_t u = 0; u < n_users; ++u) {
            deg[u] = std::min<int64_t>(cap, std::max<int64_t>(1, (int64_t)std::llround(raw[u] * scale)));
            tot += deg[u];
        }
        // exact total: adjust random users one rating at a time
        while (tot != nnz) {
            const int64_t u = (int64_t)rng.below(n_users);
            if (tot < nnz && deg[u] < cap) { ++deg[u]; ++tot; }
            else if (tot > nnz && deg[u] > 1) { --deg[u]; --tot; }
        }
    }
    // --- item popularity: w(rank) = (rank + 1 + offset)^-exponent over a seeded random rank order ---
    std::vector<double> w(n_movies);
    std::vector<int32_t> perm(n_movies);
    std::iota(perm.begin(), perm.end(), 0);
    {
        Rng rng(mix64(seed ^ sp.perm_salt));
        for (int64_t i = n_movies - 1; i > 0; --i) std::swap(perm[i], perm[rng.below(i + 1)]);
        for (int64_t r = 0; r < n_movies; ++r) w[perm[r]] = std::pow((double)(r + 1) + sp.rank_offset, -sp.exponent);
    }
    // alias table (Vose)
    std::vector<double> prob(n_movies);
    std::vector<int32_t> alias(n_movies);
    {
        const double tw = std::accumulate(w.begin(), w.end(), 0.0);
        std::vector<double> p(n_movies);
        std::vector<int32_t> small, large;
        for (int64_t i = 0; i < n_movies; ++i) {
            p[i] = w[i] * (double)n_movies / tw;
            (p[i] < 1.0 ? small : large).push_back((int32_t)i);
        }
        while (!small.empty() && !large.empty()) {
            const int32_t s = small.back(), l = large.back();
            small.pop_back();
            prob[s] = p[s];
            alias[s] = l;
            p[l] = (p[l] + p[s]) - 1.0;
            if (p[l] < 1.0) {
                large.pop_back();
                small.push_back(l);
            }
        }
        for (int32_t i : large) { prob[i] = 1.0; alias[i] = i; }
        for (int32_t i : small) { prob[i] = 1.0; alias[i] = i; }
    }
    // rating histogram of data_sample_medium.txt: 1: 4.55%, 2: 9.78%, 3: 28.37%, 4: 33.51%, 5: 23.80%
    const double cdf[5] = {0.0455, 0.0455 + 0.0978, 0.0455 + 0.0978 + 0.2837, 0.0455 + 0.0978 + 0.2837 + 0.3351, 1.0};
    // one user's distinct movies (sorted) and ratings, deterministic per user
    auto gen_user = [&](int64_t u, int32_t* dst, int16_t* rat, std::vector<int32_t>& stamp) {
        Rng rng(mix64(seed * 0x9E3779B97F4A7C15ULL + (uint64_t)u));
        const int64_t d = deg[u];
        int64_t got = 0, tries = 0;
        const int64_t max_tries = 64 * d + 100000;
        while (got < d && tries < max_tries) {
            ++tries;
            const int64_t i = (int64_t)rng.below(n_movies);
            const int32_t m = rng.uniform() < prob[i] ? (int32_t)i : alias[i];
            if (stamp[m] == (int32_t)u) continue;
            stamp[m] = (int32_t)u;
            dst[got++] = m;
        }
        for (int64_t m = (int64_t)rng.below(n_movies); got < d; m = (m + 1) % n_movies)   // fallback
            if (stamp[m] != (int32_t)u) {
                stamp[m] = (int32_t)u;
                dst[got++] = (int32_t)m;
            }
        std::sort(dst, dst + d);
        for (int64_t t = 0; t < d; ++t) {
            const double x = rng.uniform();
            int r = 0;
            while (r < 4 && x >= cdf[r]) ++r;
            rat[t] = (int16_t)(r + 1);
        }
    };
    if (G > 1) {
        // Shard-restricted: every user's list is generated (the same draws as below), only shard `keep`'s ratings are
        // kept (about 2/G of nnz instead of the whole matrix per process), plus every user's rating sum (U0) and the
        // movie degrees (the every-movie-rated guarantee, which the full path enforces with a global fix-up pass: the
        // restricted path requires that no movie is unrated, true of every configured shape: the rarest configs[4]
        // item expects ~140 ratings).
        struct Kept { int32_t m, u; int16_t r; };
        const int64_t n_chunks = (n_users + 255) / 256;
        std::vector<std::vector<Kept>> chunk(n_chunks);
        std::vector<int64_t> usum(n_users, 0), ucnt(n_users, 0);
        std::vector<std::vector<int64_t>> mdeg_t(nthreads);
        std::atomic<int64_t> next{0};
        auto worker = [&](int w) {
            std::vector<int32_t> stamp(n_movies, -1), lst;
            std::vector<int16_t> rat;
            std::vector<int64_t>& mdeg = mdeg_t[w];
            mdeg.assign(n_movies, 0);
            for (;;) {
                const int64_t c = next.fetch_add(1);
                if (c >= n_chunks) break;
                for (int64_t u = c * 256; u < std::min<int64_t>(n_users, c * 256 + 256); ++u) {
                    lst.resize(deg[u]);
                    rat.resize(deg[u]);
                    gen_user(u, lst.data(), rat.data(), stamp);
                    const bool own_user = (u + 1) % G == keep;
                    for (int64_t t = 0; t < deg[u]; ++t) {
                        ++mdeg[lst[t]];
                        usum[u] += rat[t];
                        if (own_user || (lst[t] + 1) % G == keep) chunk[c].push_back({lst[t], (int32_t)u, rat[t]});
                    }
                    ucnt[u] = deg[u];
                }
            }
        };
        std::vector<std::thread> pool;
        for (int i = 0; i < nthreads; ++i) pool.emplace_back(worker, i);
        for (auto& t : pool) t.join();
        for (int64_t m = 0; m < n_movies; ++m) {
            int64_t d = 0;
            for (auto& v : mdeg_t) d += v[m];
            if (d == 0)
                return report(fail(ALS_ERR_UNSUPPORTED, "movie %lld unrated: the shard-restricted generator needs every "
                                   "movie rated (use the full generator)", (long long)m + 1));
        }
        mdeg_t.clear();
        // movie-major arrival order: stable counting sort by movie of the user-major kept ratings
        std::unique_ptr<als_dataset> ds(new als_dataset());
        std::vector<int64_t> moff(n_movies + 1, 0);
        int64_t kept = 0;
        for (auto& ch : chunk) {
            kept += (int64_t)ch.size();
            for (const Kept& k : ch) ++moff[k.m + 1];
        }
        for (int64_t m = 0; m < n_movies; ++m) moff[m + 1] += moff[m];
        ds->movie.resize(kept);
        ds->user.resize(kept);
        ds->rating.resize(kept);
        std::vector<int64_t> pos(moff.begin(), moff.end() - 1);
        for (auto& ch : chunk) {
            for (const Kept& k : ch) {
                const int64_t p = pos[k.m]++;
                ds->movie[p] = k.m + 1;
                ds->user[p] = k.u + 1;
                ds->rating[p] = k.r;
            }
            std::vector<Kept>().swap(ch);
        }
        ds->ids[0].resize(n_movies);
        ds->ids[1].resize(n_users);
        std::iota(ds->ids[0].begin(), ds->ids[0].end(), 1);
        std::iota(ds->ids[1].begin(), ds->ids[1].end(), 1);
        ds->dense[0].resize(kept);
        ds->dense[1].resize(kept);
        for (int64_t t = 0; t < kept; ++t) {
            ds->dense[0][t] = ds->movie[t] - 1;
            ds->dense[1][t] = ds->user[t] - 1;
        }
        ds->user_sum.swap(usum);
        ds->user_cnt.swap(ucnt);
        *out = ds.release();
        return ALS_OK;
    }
    // --- per-user distinct movie lists (user-major), deterministic per user ---
    std::vector<int64_t> uoff(n_users + 1, 0);
    for (int64_t u = 0; u < n_users; ++u) uoff[u + 1] = uoff[u] + deg[u];
    std::vector<int32_t> um(nnz);
    std::vector<int16_t> ur(nnz);
    {
        std::atomic<int64_t> next_user{0};
        auto worker = [&]() {
            std::vector<int32_t> stamp(n_movies, -1);
            for (;;) {
                const int64_t u0 = next_user.fetch_add(256);
                if (u0 >= n_users) break;
                const int64_t u1 = std::min<int64_t>(n_users, u0 + 256);
                for (int64_t u = u0; u < u1; ++u) gen_user(u, um.data() + uoff[u], ur.data() + uoff[u], stamp);
            }
        };
        std::vector<std::thread> pool;
        for (int i = 0; i < nthreads; ++i) pool.emplace_back(worker);
        for (auto& t : pool) t.join();
    }
    // --- every movie rated at least once: re-point one entry of a popular movie (keeps nnz exact) ---
    {
        std::vector<int64_t> mdeg(n_movies, 0);
        for (int64_t t = 0; t < nnz; ++t) ++mdeg[um[t]];
        Rng rng(mix64(seed ^ 0xF111ULL));
        for (int64_t m = 0; m < n_movies; ++m) {
            if (mdeg[m] > 0) continue;
            for (;;) {
                const int64_t t = (int64_t)rng.below(nnz);
                if (mdeg[um[t]] < 2) continue;
                // owning user of entry t
                const int64_t u = (int64_t)(std::upper_bound(uoff.begin(), uoff.end(), t) - uoff.begin()) - 1;
                const int32_t* b = um.data() + uoff[u];
                const int32_t* e = um.data() + uoff[u + 1];
                if (std::binary_search(b, e, (int32_t)m)) continue;
                --mdeg[um[t]];
                um[t] = (int32_t)m;
                ++mdeg[m];
                std::sort(um.data() + uoff[u], um.data() + uoff[u + 1]);   // keep the row sorted (ratings stay iid)
                break;
            }
        }
    }
    // --- movie-major arrival order (stable counting sort by movie; users ascending inside a movie) ---
    std::unique_ptr<als_dataset> ds(new als_dataset());
    {
        std::vector<int64_t> moff(n_movies + 1, 0);
        for (int64_t t = 0; t < nnz; ++t) ++moff[um[t] + 1];
        for (int64_t m = 0; m < n_movies; ++m) moff[m + 1] += moff[m];
        ds->movie.resize(nnz);
        ds->user.resize(nnz);
        ds->rating.resize(nnz);
        std::vector<int64_t> pos(moff.begin(), moff.end() - 1);
        for (int64_t u = 0; u < n_users; ++u)
            for (int64_t t = uoff[u]; t < uoff[u + 1]; ++t) {
                const int64_t p = pos[um[t]]++;
                ds->movie[p] = um[t] + 1;
                ds->user[p] = (int32_t)(u + 1);
                ds->rating[p] = ur[t];
            }
        // dense ranks are known directly: ids are 1..n and every entity is rated
        ds->ids[0].resize(n_movies);
        ds->ids[1].resize(n_users);
        std::iota(ds->ids[0].begin(), ds->ids[0].end(), 1);
        std::iota(ds->ids[1].begin(), ds->ids[1].end(), 1);
        ds->dense[0].resize(nnz);
        ds->dense[1].resize(nnz);
        for (int64_t t = 0; t < nnz; ++t) {
            ds->dense[0][t] = ds->movie[t] - 1;
            ds->dense[1][t] = ds->user[t] - 1;
        }
    }
    *out = ds.release();
    return ALS_OK;
}

}  // namespace

extern "C" {

int als_dataset_synthetic_netflix(int64_t n_users, int64_t n_movies, int64_t nnz, uint64_t seed, int nthreads,
                                  als_dataset** out) {
    // user degrees log-normal (median 96, mean 208.2 at Netflix scale, cap 17,653); movies (rank + 320)^-1.85
    const SynthSpec sp{std::log(96.0), std::sqrt(2.0 * std::log(208.2 / 96.0)), 17653, 320.0, 1.85, 0x30F1EULL};
    return synthesize(sp, n_users, n_movies, nnz, seed, nthreads, out);
}

int als_dataset_synthetic_powerlaw(int64_t n_users, int64_t n_items, int64_t nnz, uint64_t seed, int nthreads,
                                   als_dataset** out) {
    // user activity log-normal with sigma 1.5 and mean nnz / n_users; item popularity ~ rank^-1 (Zipf);
    // per-user cap n_items / 10 (the heaviest users and items are the load-balance stress)
    const double sigma = 1.5, mean = (double)nnz / (double)std::max<int64_t>(1, n_users);
    const SynthSpec sp{std::log(mean) - 0.5 * sigma * sigma, sigma, std::max<int64_t>(1, n_items / 10), 0.0, 1.0,
                       0x9A11ULL};
    return synthesize(sp, n_users, n_items, nnz, seed, nthreads, out);
}

int als_dataset_synthetic_powerlaw_shard(int64_t n_users, int64_t n_items, int64_t nnz, uint64_t seed, int nthreads,
                                         int n_shards, int shard, als_dataset** out) {
    const double sigma = 1.5, mean = (double)nnz / (double)std::max<int64_t>(1, n_users);
    const SynthSpec sp{std::log(mean) - 0.5 * sigma * sigma, sigma, std::max<int64_t>(1, n_items / 10), 0.0, 1.0,
                       0x9A11ULL};
    return synthesize(sp, n_users, n_items, nnz, seed, nthreads, out, n_shards, shard);
}

int als_dataset_synthetic_netflix_shard(int64_t n_users, int64_t n_movies, int64_t nnz, uint64_t seed, int nthreads,
                                        int n_shards, int shard, als_dataset** out) {
    const SynthSpec sp{std::log(96.0), std::sqrt(2.0 * std::log(208.2 / 96.0)), 17653, 320.0, 1.85, 0x30F1EULL};
    return synthesize(sp, n_users, n_movies, nnz, seed, nthreads, out, n_shards, shard);
}

int als_dataset_destroy(als_dataset* ds) {
    delete ds;
    return ALS_OK;
}

int als_dataset_counts(const als_dataset* ds, int64_t* n_movies, int64_t* n_users, int64_t* nnz) {
    if (!ds) return report(fail(ALS_ERR_INVALID_ARGUMENT, "dataset is NULL"));
    if (n_movies) *n_movies = (int64_t)ds->ids[0].size();
    if (n_users) *n_users = (int64_t)ds->ids[1].size();
    if (nnz) *nnz = (int64_t)ds->rating.size();
    return ALS_OK;
}

int als_dataset_ids(const als_dataset* ds, int side, int64_t* ids) {
    if (!ds || (side != 0 && side != 1) || !ids) return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    std::copy(ds->ids[side].begin(), ds->ids[side].end(), ids);
    return ALS_OK;
}

int als_dataset_ratings(const als_dataset* ds, int32_t* movie_ids, int32_t* user_ids, int16_t* ratings) {
    if (!ds) return report(fail(ALS_ERR_INVALID_ARGUMENT, "dataset is NULL"));
    if (movie_ids) std::copy(ds->movie.begin(), ds->movie.end(), movie_ids);
    if (user_ids) std::copy(ds->user.begin(), ds->user.end(), user_ids);
    if (ratings) std::copy(ds->rating.begin(), ds->rating.end(), ratings);
    return ALS_OK;
}

int als_dataset_count_duplicates(const als_dataset* ds, int64_t* n_dup) {
    if (!ds || !n_dup) return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const int64_t n = (int64_t)ds->rating.size();
    std::vector<uint64_t> key(n);
    for (int64_t t = 0; t < n; ++t) key[t] = ((uint64_t)(uint32_t)ds->dense[1][t] << 32) | (uint32_t)ds->dense[0][t];
    std::sort(key.begin(), key.end());
    int64_t d = 0;
    for (int64_t t = 1; t < n; ++t) d += key[t] == key[t - 1];
    *n_dup = d;
    return ALS_OK;
}

int als_dataset_shard_info(const als_dataset* ds, int side, int n_shards, int shard, int64_t* n_rows,
                           int64_t* row_offset, int64_t* nnz, int64_t* slots_per_shard, int64_t* n_slots) {
    if (!ds || (side != 0 && side != 1) || n_shards < 1 || shard < 0 || shard >= n_shards)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const ShardMap m = shard_map(ds, side, n_shards);
    int64_t z = 0;
    const auto& raw = side == 0 ? ds->movie : ds->user;
    for (int32_t v : raw) z += (v % n_shards) == shard;
    if (n_rows) *n_rows = m.count[shard];
    if (row_offset) *row_offset = shard * m.Sc;
    if (nnz) *nnz = z;
    if (slots_per_shard) *slots_per_shard = m.Sc * m.C;
    if (n_slots) *n_slots = m.n_slots();
    return ALS_OK;
}

int als_dataset_set_slot_chunks(als_dataset* ds, int side, int n_chunks) {
    if (!ds || (side != 0 && side != 1) || n_chunks < 1) return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    ds->chunks[side] = n_chunks;
    return ALS_OK;
}

int als_dataset_slot_layout(const als_dataset* ds, int side, int n_shards, int64_t* slots_per_chunk, int* n_chunks) {
    if (!ds || (side != 0 && side != 1) || n_shards < 1) return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const ShardMap m = shard_map(ds, side, n_shards);
    if (slots_per_chunk) *slots_per_chunk = m.Sc;
    if (n_chunks) *n_chunks = m.C;
    return ALS_OK;
}

int als_dataset_shard_block(const als_dataset* ds, int side, int n_shards, int64_t shard, int64_t* row_ptr,
                            int32_t* col_idx, int16_t* ratings, int64_t* row_ids) {
    if (!ds || (side != 0 && side != 1) || n_shards < 1 || shard < 0 || shard >= n_shards || !row_ptr)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const int opp = 1 - side;
    const ShardMap ms = shard_map(ds, side, n_shards);
    const ShardMap mo = shard_map(ds, opp, n_shards);
    const int64_t nr = ms.count[shard];
    const auto& dn = ds->dense[side];
    const auto& dop = ds->dense[opp];
    const int64_t n = (int64_t)dn.size();
    // stable counting sort of arrival order by local row: in-block order = arrival order
    std::fill(row_ptr, row_ptr + nr + 1, 0);
    for (int64_t t = 0; t < n; ++t)
        if (ms.shard[dn[t]] == shard) ++row_ptr[ms.local[dn[t]] + 1];
    for (int64_t i = 0; i < nr; ++i) row_ptr[i + 1] += row_ptr[i];
    if (col_idx || ratings) {
        std::vector<int64_t> pos(row_ptr, row_ptr + nr);
        for (int64_t t = 0; t < n; ++t) {
            if (ms.shard[dn[t]] != shard) continue;
            const int64_t p = pos[ms.local[dn[t]]]++;
            if (col_idx) col_idx[p] = (int32_t)mo.slot[dop[t]];
            if (ratings) ratings[p] = ds->rating[t];
        }
    }
    if (row_ids) {
        const auto& ids = ds->ids[side];
        for (size_t i = 0; i < ids.size(); ++i)
            if (ms.shard[i] == shard) row_ids[ms.local[i]] = ids[i];
    }
    return ALS_OK;
}

int als_dataset_shard_coo(const als_dataset* ds, int side, int n_shards, int64_t shard, int32_t* rows,
                          int32_t* cols, int16_t* ratings) {
    if (!ds || (side != 0 && side != 1) || n_shards < 1 || shard < 0 || shard >= n_shards || !rows || !cols || !ratings)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const int opp = 1 - side;
    const ShardMap ms = shard_map(ds, side, n_shards);
    const ShardMap mo = shard_map(ds, opp, n_shards);
    const auto& dn = ds->dense[side];
    const auto& dop = ds->dense[opp];
    const int64_t n = (int64_t)dn.size();
    int64_t p = 0;
    for (int64_t t = 0; t < n; ++t) {   // arrival order: the order the block builder sees the ratings
        if (ms.shard[dn[t]] != shard) continue;
        rows[p] = (int32_t)ms.local[dn[t]];
        cols[p] = (int32_t)mo.slot[dop[t]];
        ratings[p] = ds->rating[t];
        ++p;
    }
    return ALS_OK;
}

int als_dataset_slots(const als_dataset* ds, int side, int n_shards, int64_t* slot_of) {
    if (!ds || (side != 0 && side != 1) || n_shards < 1 || !slot_of)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const ShardMap m = shard_map(ds, side, n_shards);
    std::copy(m.slot.begin(), m.slot.end(), slot_of);
    return ALS_OK;
}

int als_dataset_init_user_factors(const als_dataset* ds, int num_features, uint64_t seed, int n_shards, float* out,
                                  int64_t ld, int64_t n_out_rows) {
    if (!ds || num_features < 1 || n_shards < 1 || !out || ld < num_features)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    const ShardMap m = shard_map(ds, 1, n_shards);
    if (n_out_rows < m.n_slots()) return report(fail(ALS_ERR_INVALID_ARGUMENT, "output has too few rows"));
    std::fill(out, out + n_out_rows * ld, 0.f);
    const int64_t nu = (int64_t)ds->ids[1].size();
    std::vector<int64_t> sum(nu, 0), cnt(nu, 0);
    if (!ds->user_cnt.empty()) {   // shard-restricted synthetic data: the full sums were kept at generation
        sum = ds->user_sum;
        cnt = ds->user_cnt;
    } else {
        for (size_t t = 0; t < ds->rating.size(); ++t) {
            sum[ds->dense[1][t]] += ds->rating[t];
            ++cnt[ds->dense[1][t]];
        }
    }
    for (int64_t u = 0; u < nu; ++u) {
        float* f = out + m.slot[u] * ld;
        // DoubleStream.average() (exact for short ratings) cast to float; orElse(1.0)
        const double mean = cnt[u] > 0 ? (double)sum[u] / (double)cnt[u] : 1.0;
        f[0] = (float)mean;
        for (int c = 1; c < num_features; ++c) f[c] = als_u01(seed, ds->ids[1][u], c);
    }
    return ALS_OK;
}

}  // extern "C"

namespace {

// EJML MatrixIO.saveDenseCSV of the widened matrix; cell(i, j) yields the fp32 prediction.
template <class Cell>
int write_csv(const char* path, int64_t n_users, int64_t n_movies, Cell cell) {
    FILE* f = fopen(path, "wb");
    if (!f) return report(fail(ALS_ERR_IO, "cannot create %s", path));
    fprintf(f, "%lld %lld real\n", (long long)n_users, (long long)n_movies);
    std::string line;
    for (int64_t i = 0; i < n_users; ++i) {
        line.clear();
        for (int64_t j = 0; j < n_movies; ++j) {
            line += java_double((double)cell(i, j));
            line.push_back(' ');
        }
        line.push_back('\n');
        if (fwrite(line.data(), 1, line.size(), f) != line.size()) {
            fclose(f);
            return report(fail(ALS_ERR_IO, "write failed: %s", path));
        }
    }
    if (fclose(f) != 0) return report(fail(ALS_ERR_IO, "close failed: %s", path));
    return ALS_OK;
}

}  // namespace

extern "C" {

int als_write_prediction_csv(const char* path, const float* U, int64_t n_users, int64_t ldu, const float* M,
                             int64_t n_movies, int64_t ldm, int num_features) {
    if (!path || (n_users > 0 && !U) || (n_movies > 0 && !M) || num_features < 1 || ldu < num_features ||
        ldm < num_features)
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    return write_csv(path, n_users, n_movies, [&](int64_t i, int64_t j) {
        const float* x = U + i * ldu;
        const float* y = M + j * ldm;
        float total = 0.f;   // MatrixMatrixMult_FDRM.multTransB: sequential fp32 dot
        for (int c = 0; c < num_features; ++c) total += x[c] * y[c];
        return total;
    });
}

int als_write_prediction_matrix_csv(const char* path, const float* P, int64_t n_users, int64_t n_movies) {
    if (!path || n_users < 0 || n_movies < 0 || (n_users > 0 && n_movies > 0 && !P))
        return report(fail(ALS_ERR_INVALID_ARGUMENT, "bad arguments"));
    return write_csv(path, n_users, n_movies, [&](int64_t i, int64_t j) { return P[i * n_movies + j]; });
}

}  // extern "C"
