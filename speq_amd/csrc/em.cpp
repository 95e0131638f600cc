// Host half of the EM refinement: histogram rows and the EM step (see em.hpp).
#include "em.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <limits>
#include <mutex>
#include <thread>

#include "scan_internal.hpp"

namespace {
constexpr uint64_t EM_CHUNKS = 64;  // fixed row partition of speq_em_step (deterministic across machines)

// Workers of speq_em_step, started once per process: a step takes 1-2 ms, and starting 16 threads for every one of
// a run's 20-30 steps cost about as much as the sweep. run(n, f) calls f(0..n-1) on the workers and the caller.
class StepPool {
public:
    explicit StepPool(uint32_t n) : workers_(n) {
        for (uint32_t i = 0; i < n; ++i)
            ws_.emplace_back([this] {
                uint64_t seen = 0;
                for (;;) {
                    {
                        std::unique_lock<std::mutex> lk(mu_);
                        cv_.wait(lk, [&] { return gen_ != seen; });
                        seen = gen_;
                    }
                    drain();
                    std::lock_guard<std::mutex> lk(mu_);
                    if (--pending_ == 0) done_.notify_all();
                }
            });
    }
    // every worker takes part in every run (so none can still be in this one when the next begins)
    void run(uint64_t n, const std::function<void(uint64_t)>& f) {
        std::lock_guard<std::mutex> one(run_mu_);  // (one step at a time in the process)
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &f;
            n_ = n;
            next_ = 0;
            pending_ = workers_;
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return pending_ == 0; });
    }

private:
    void drain() {
        for (uint64_t i; (i = next_.fetch_add(1)) < n_;) (*job_)(i);
    }
    const uint32_t workers_;
    std::vector<std::thread> ws_;  // (never joined: the pool lives until the process ends)
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    const std::function<void(uint64_t)>* job_ = nullptr;
    std::atomic<uint64_t> next_{0};
    uint64_t n_ = 0, gen_ = 0;
    uint32_t pending_ = 0;
};

StepPool& step_pool() {
    static StepPool* p = new StepPool(std::min(std::max(1u, std::thread::hardware_concurrency()), 16u) - 1u);
    return *p;
}
}  // namespace

namespace speq {

// Rows with the same (group, count) entries — k-mers whose occurrences lie in the same texts — contribute the same
// function of the step's percentages times their multiplicity, so they are merged into the first of them with the
// multiplicities summed (the sums then differ from row-by-row ones by fp64 re-association only). Row order: first
// occurrence. SPEQ_EM_MERGE_ROWS=0 keeps every interval's row (A/B).
void merge_equal_rows(speq_em& em) {
    const char* e = std::getenv("SPEQ_EM_MERGE_ROWS");
    const uint64_t R = em.row_mult.size();
    if ((e && e[0] == '0') || R < 2) return;
    std::vector<uint64_t> h(R);
    const uint64_t n_chunks = std::min<uint64_t>(EM_CHUNKS, std::max<uint64_t>(1, R / 2048));
    auto hash_rows = [&](uint64_t ci) {
        for (uint64_t r = R * ci / n_chunks; r < R * (ci + 1) / n_chunks; ++r) {
            uint64_t x = 0x9E3779B97F4A7C15ull ^ (em.row_ptr[r + 1] - em.row_ptr[r]);
            for (uint64_t i = em.row_ptr[r]; i < em.row_ptr[r + 1]; ++i) {
                x ^= ((uint64_t)em.col_group[i] << 32) | em.col_count[i];
                x *= 0xFF51AFD7ED558CCDull;
                x ^= x >> 29;
            }
            h[r] = x;
        }
    };
    if (n_chunks <= 1) hash_rows(0);
    else step_pool().run(n_chunks, hash_rows);
    auto same = [&](uint64_t a, uint64_t b) {
        const uint64_t na = em.row_ptr[a + 1] - em.row_ptr[a];
        if (na != em.row_ptr[b + 1] - em.row_ptr[b]) return false;
        return std::equal(em.col_group.begin() + em.row_ptr[a], em.col_group.begin() + em.row_ptr[a + 1],
                          em.col_group.begin() + em.row_ptr[b]) &&
               std::equal(em.col_count.begin() + em.row_ptr[a], em.col_count.begin() + em.row_ptr[a + 1],
                          em.col_count.begin() + em.row_ptr[b]);
    };
    // open addressing over the hashes: slot -> 1 + the first row with that content. First by hash alone, each row's
    // representative then checked entry by entry (in parallel); a hash collision between different contents (never
    // seen) redoes the assignment comparing entries.
    uint64_t cap = 1;
    while (cap < 2 * R) cap <<= 1;
    std::vector<uint64_t> rep(R);
    uint64_t distinct = 0;
    auto assign = [&](bool exact) {
        std::vector<uint64_t> slot(cap, 0);
        distinct = 0;
        for (uint64_t r = 0; r < R; ++r) {
            for (uint64_t s = h[r] & (cap - 1);; s = (s + 1) & (cap - 1)) {
                if (slot[s] == 0) {
                    slot[s] = r + 1;
                    rep[r] = r;
                    ++distinct;
                    break;
                }
                const uint64_t q = slot[s] - 1;
                if (h[q] == h[r] && (!exact || same(q, r))) {
                    rep[r] = q;
                    break;
                }
            }
        }
    };
    assign(false);
    std::atomic<bool> collided{false};
    auto verify = [&](uint64_t ci) {
        for (uint64_t r = R * ci / n_chunks; r < R * (ci + 1) / n_chunks; ++r)
            if (rep[r] != r && !same(rep[r], r)) collided = true;
    };
    if (n_chunks <= 1) verify(0);
    else step_pool().run(n_chunks, verify);
    if (collided) assign(true);
    if (distinct == R) return;
    std::vector<uint64_t> at(R), mult, ptr(1, 0);
    std::vector<uint32_t> grp, cnt;
    mult.reserve(distinct);
    ptr.reserve(distinct + 1);
    for (uint64_t r = 0; r < R; ++r) {
        if (rep[r] != r) {
            mult[at[rep[r]]] += em.row_mult[r];
            continue;
        }
        at[r] = mult.size();
        mult.push_back(em.row_mult[r]);
        grp.insert(grp.end(), em.col_group.begin() + em.row_ptr[r], em.col_group.begin() + em.row_ptr[r + 1]);
        cnt.insert(cnt.end(), em.col_count.begin() + em.row_ptr[r], em.col_count.begin() + em.row_ptr[r + 1]);
        ptr.push_back(grp.size());
    }
    em.row_mult.swap(mult);
    em.row_ptr.swap(ptr);
    em.col_group.swap(grp);
    em.col_count.swap(cnt);
}

void em_build_rows(speq_em& em, const uint32_t* lo, const uint32_t* mult, const uint32_t* hi, uint64_t m) {
    const FmIndex& fm = em.idx->fm;
    // contiguous chunks of intervals, built on the step pool's workers and appended in chunk order (rows in lo order)
    const uint64_t n_chunks = std::min<uint64_t>(EM_CHUNKS, std::max<uint64_t>(1, m / 2048));
    struct Part {
        std::vector<uint64_t> mult, nnz;
        std::vector<uint32_t> grp, cnt;
    };
    std::vector<Part> parts(n_chunks);
    const bool lab = !fm.lab.empty();
    auto build = [&](uint64_t ci) {
        Part& P = parts[ci];
        std::vector<uint32_t> dense(em.G, 0);
        std::vector<uint32_t> touched;
        const uint64_t b = m * ci / n_chunks, e = m * (ci + 1) / n_chunks;
        P.mult.reserve(e - b);
        P.nnz.reserve(e - b);
        for (uint64_t r = b; r < e; ++r) {
            const uint64_t h = hi[r];
            // per-group occurrence counts c_g = overlap of [lo, h) with the label runs of group g; the label table
            // gives a run's group and its distance to the run's end in one load (saturated distances: the rank path)
            for (uint64_t i = lo[r]; i < h;) {
                uint64_t j;
                uint16_t g;
                const uint32_t x = lab ? fm.lab[i] : 0u;
                if (lab && (x >> 16) != 0xFFFFu) {
                    g = (uint16_t)(x & 0xFFFFu);
                    j = std::min<uint64_t>(i + (x >> 16), h);
                } else {
                    g = fm.label_at(i);
                    j = std::min<uint64_t>(fm.run_end(i), h);
                }
                if (!dense[g]) touched.push_back(g);
                dense[g] += (uint32_t)(j - i);
                i = j;
            }
            std::sort(touched.begin(), touched.end());  // the reference sums groups in index order
            P.mult.push_back(mult[r]);
            P.nnz.push_back(touched.size());
            for (uint32_t g : touched) {
                P.grp.push_back(g);
                P.cnt.push_back(dense[g]);
                dense[g] = 0;
            }
            touched.clear();
        }
    };
    if (n_chunks <= 1) {
        build(0);
    } else {
        step_pool().run(n_chunks, build);
    }
    uint64_t rows = 0, ents = 0;
    for (const Part& P : parts) {
        rows += P.mult.size();
        ents += P.grp.size();
    }
    em.row_mult.clear();
    em.row_mult.reserve(rows);
    em.row_ptr.assign(1, 0);
    em.row_ptr.reserve(rows + 1);
    em.col_group.clear();
    em.col_group.reserve(ents);
    em.col_count.clear();
    em.col_count.reserve(ents);
    for (auto& P : parts) {
        em.row_mult.insert(em.row_mult.end(), P.mult.begin(), P.mult.end());
        for (uint64_t z : P.nnz) em.row_ptr.push_back(em.row_ptr.back() + z);
        em.col_group.insert(em.col_group.end(), P.grp.begin(), P.grp.end());
        em.col_count.insert(em.col_count.end(), P.cnt.begin(), P.cnt.end());
    }
    em.n_intervals = em.row_mult.size();
    em.n_entries = em.col_group.size();
    merge_equal_rows(em);
    char msg[96];
    std::snprintf(msg, sizeof msg, "em rows: %llu intervals -> %llu rows",
                  (unsigned long long)em.n_intervals, (unsigned long long)em.row_mult.size());
    startup_trace(msg);
    em.finalized = true;
}

}  // namespace speq

extern "C" {

int speq_em_info(const speq_em* em, uint64_t* n_intervals, uint64_t* n_entries, uint64_t* n_windows) {
    return speq::guarded([&] {
        if (!em || !em->finalized) throw std::invalid_argument("speq_em_info: histogram not finalized");
        if (n_intervals) *n_intervals = em->n_intervals;
        if (n_entries) *n_entries = em->n_entries;
        if (n_windows) {
            uint64_t s = 0;
            for (uint64_t m : em->row_mult) s += m;
            *n_windows = s;
        }
    });
}

// One EM step (fm_scanner.cpp:1098-1120 global, :1186-1214 local): for every passing window with hits,
// a_i = c_i p_i / n_i, norm = sum_i a_i (group order), and if norm > 0, next_i += a_i / norm.
int speq_em_step(const speq_em* em, const double* percent, const int32_t* group_counts, const uint64_t* unique,
                 double* next) {
    return speq::guarded([&] {
        if (!em || !percent || !group_counts || !unique || !next) throw std::invalid_argument("speq_em_step: null argument");
        if (!em->finalized) throw std::invalid_argument("speq_em_step: histogram not finalized");
        const uint32_t G = em->G;
        std::vector<double> coef(G);  // p_i / n_i, evaluated as (c * p) / n below
        bool clean = true;            // every "0 * p_i / n_i" term is exactly 0 (no n_i == 0, finite p_i)
        for (uint32_t g = 0; g < G; ++g) {
            const double z = 0.0 * percent[g] / (double)group_counts[g];
            if (!(z == 0.0)) clean = false;
        }
        std::fill(next, next + G, 0.0);
        const uint64_t R = em->row_mult.size();
        if (clean) {
            // single-group windows: a / a = 1 when a = c p_g / n_g > 0 (c >= 1), else norm == 0 and they are skipped
            for (uint32_t g = 0; g < G; ++g) {
                const double a = percent[g] / (double)group_counts[g];
                if (a > 0.0) next[g] += (double)unique[g];
            }
            // Rows are split into a FIXED number of contiguous chunks (independent of the machine's thread count),
            // each summed into its own vector, and the chunk vectors are added in chunk order: the result is
            // deterministic, and differs from a serial sweep only by fp64 re-association (tests: rtol 1e-9).
            const uint64_t n_chunks = std::min<uint64_t>(EM_CHUNKS, std::max<uint64_t>(1, em->col_group.size() / 16384));
            std::vector<double> part(n_chunks * G, 0.0);
            auto run_chunk = [&](uint64_t ci) {
                const uint64_t r0 = R * ci / n_chunks, r1 = R * (ci + 1) / n_chunks;
                double* acc = part.data() + ci * G;
                std::vector<double> a;
                for (uint64_t r = r0; r < r1; ++r) {
                    const uint64_t b = em->row_ptr[r], e = em->row_ptr[r + 1];
                    a.resize(e - b);
                    double norm = 0.0;
                    for (uint64_t x = b; x < e; ++x) {
                        const uint32_t g = em->col_group[x];
                        a[x - b] = (double)em->col_count[x] * percent[g] / (double)group_counts[g];
                        norm += a[x - b];
                    }
                    if (norm > 0.0) {
                        const double m = (double)em->row_mult[r];
                        for (uint64_t x = b; x < e; ++x) acc[em->col_group[x]] += m * (a[x - b] / norm);
                    }
                }
            };
            if (n_chunks <= 1) {
                run_chunk(0);
            } else {
                step_pool().run(n_chunks, run_chunk);
            }
            for (uint64_t ci = 0; ci < n_chunks; ++ci)
                for (uint32_t g = 0; g < G; ++g) next[g] += part[ci * G + g];
        } else {
            // IEEE edge cases (a group count of 0, non-finite percentages): evaluate every group of every row
            // exactly as the reference does, zero terms included.
            std::vector<double> a(G);
            auto window = [&](const uint32_t* grp, const uint32_t* cnt, uint64_t nnz, double m) {
                std::vector<double> h(G, 0.0);
                for (uint64_t x = 0; x < nnz; ++x) h[grp[x]] = (double)cnt[x];
                double norm = 0.0;
                for (uint32_t g = 0; g < G; ++g) {
                    a[g] = h[g] * percent[g] / (double)group_counts[g];
                    norm += a[g];
                }
                if (norm > 0.0)
                    for (uint32_t g = 0; g < G; ++g) next[g] += m * (a[g] / norm);
            };
            for (uint32_t g = 0; g < G; ++g) {
                if (!unique[g]) continue;
                const uint32_t one = 1;
                window(&g, &one, 1, (double)unique[g]);
            }
            for (uint64_t r = 0; r < R; ++r) {
                const uint64_t b = em->row_ptr[r];
                window(em->col_group.data() + b, em->col_count.data() + b, em->row_ptr[r + 1] - b,
                       (double)em->row_mult[r]);
            }
        }
    });
}

}  // extern "C"
