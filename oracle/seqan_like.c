/*
 * seqan_like.c — a CPU stand-in for the REFERENCE'S ALGORITHM (SeqAn 3.0.1 fm_index + search + locate).
 * TEST / BASELINE INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's cpu_baseline leg, never by speq_amd/.
 *
 * The reference cannot be built here (deps/seqan3 is an empty submodule; SDSL, cereal, range-v3 absent —
 * SURVEY.md §8(c)), so SURVEY.md §8(d) asks for a "SeqAn-like" CPU path as the faithful baseline: the same work
 * per window as the reference's `search(f_kmers, fm_index, cfg)` with `output{text_position}` followed by
 * `do_a_count` (src/fm_scanner.cpp:139-140, :153-196, :208):
 *
 *   1. backward search of the k-mer on a wavelet structure over the BWT (SeqAn 3.0.1's default index is
 *      sdsl::csa_wt<wt_blcd<...>, 16, 10'000'000, sa_order_sa_sampling, isa_sampling> — upstream, believed):
 *      here a 3-level wavelet matrix over the 7-symbol BWT, one rank per level per bound;
 *   2. locate of EVERY occurrence through SA samples taken every 16 SA rows (LF walks until a sampled row);
 *   3. (text_id, pos) per hit, the hit list sorted (SeqAn 3.0.x returns hits sorted by (text_id, pos));
 *   4. the reference's per-window loop over the hit list: first-hit group rule (:165-177), tallies (:164, :180),
 *      Phred weight (:454), ambiguity (:183-190; paired :709-729).
 *
 * It shares no code with the product FM-index (own suffix sorter, own rank structure, no label runs). Besides
 * timing the reference algorithm, it is a third independent restatement that tests cross-check against the
 * golden vectors and the hash-map oracle (kmer_oracle.c).
 *
 * Texts: [fwd_r, revcomp(fwd_r)] per record (src/fm_indexer.cpp:25-33), concatenated as t_0 $ t_1 $ ... #.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

#ifdef _OPENMP
#include <omp.h>
#endif

enum { S_TERM = 0, S_SEP = 1, S_A = 2, S_C = 3, S_G = 4, S_T = 5, S_N = 6, SIGMA = 7, LEVELS = 3, SAMPLE = 16 };

typedef struct {
    uint64_t* bits;   /* n bits */
    uint32_t* cum;    /* ones before word w */
    uint32_t zeros;   /* total zeros */
} level_t;

typedef struct {
    uint32_t n, n_texts, n_groups;
    level_t lv[LEVELS];
    uint32_t C[SIGMA + 1];
    uint32_t base[SIGMA];  /* position of symbol c's block after the last level (rank origin) */
    uint32_t* samples;     /* SA[16 j] */
    uint32_t* text_start;  /* n_texts + 1 */
    int32_t* text_group;
} sl_t;

static uint8_t code_of(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return S_A;
        case 'C': case 'c': return S_C;
        case 'G': case 'g': return S_G;
        case 'T': case 't': case 'U': case 'u': return S_T;
        default: return S_N;
    }
}
static uint8_t comp_code(uint8_t c) { return c == S_N ? S_N : (uint8_t)(S_T + S_A - c); }

static inline uint32_t rank1(const level_t* L, uint32_t i) {
    uint32_t w = i >> 6, b = i & 63;
    uint32_t r = L->cum[w];
    if (b) r += (uint32_t)__builtin_popcountll(L->bits[w] << (64 - b));
    return r;
}
static inline int bit_at(const level_t* L, uint32_t i) { return (int)((L->bits[i >> 6] >> (i & 63)) & 1); }

/* Maps position i through the levels for symbol c (wavelet matrix rank walk). */
static inline uint32_t wm_map(const sl_t* s, uint8_t c, uint32_t i) {
    for (int l = 0; l < LEVELS; ++l) {
        const level_t* L = &s->lv[l];
        int b = (c >> (LEVELS - 1 - l)) & 1;
        uint32_t o = rank1(L, i);
        i = b ? L->zeros + o : i - o;
    }
    return i;
}
/* LF(c, i) = C[c] + rank_c(BWT, i) */
static inline uint32_t lf(const sl_t* s, uint8_t c, uint32_t i) { return s->C[c] + wm_map(s, c, i) - s->base[c]; }

/* Reads BWT[i] and returns LF(i) in one walk. */
static inline uint32_t access_lf(const sl_t* s, uint32_t i, uint8_t* sym) {
    uint8_t c = 0;
    for (int l = 0; l < LEVELS; ++l) {
        const level_t* L = &s->lv[l];
        int b = bit_at(L, i);
        uint32_t o = rank1(L, i);
        i = b ? L->zeros + o : i - o;
        c = (uint8_t)((c << 1) | b);
    }
    *sym = c;
    return s->C[c] + i - s->base[c];
}

static uint32_t locate(const sl_t* s, uint32_t i) {
    uint32_t steps = 0;
    while (i % SAMPLE) {
        uint8_t c;
        uint32_t j = access_lf(s, i, &c);
        if (c == S_TERM) return steps;  /* SA[i] == 0 */
        i = j;
        ++steps;
    }
    return s->samples[i / SAMPLE] + steps;
}

/* ---- suffix array by prefix doubling with counting sorts (O(n log n)); independent of the product's SA-IS ---- */
static uint32_t* build_sa(const uint8_t* t, uint32_t n) {
    uint32_t* sa = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* tmp = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* rk = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t* nrk = (uint32_t*)malloc(sizeof(uint32_t) * n);
    uint32_t m = SIGMA + 1;
    uint32_t* cnt = (uint32_t*)malloc(sizeof(uint32_t) * (n > m ? n + 1 : m + 1));
    for (uint32_t i = 0; i < n; ++i) rk[i] = t[i] + 1;  /* ranks >= 1; 0 = past the end */
    for (uint32_t h = 1;; h <<= 1) {
        /* sort by (rk[i], rk[i+h]) : counting sort by second key, then stable by first key */
        memset(cnt, 0, sizeof(uint32_t) * (m + 1));
        for (uint32_t i = 0; i < n; ++i) cnt[i + h < n ? rk[i + h] : 0]++;
        for (uint32_t r = 1; r <= m; ++r) cnt[r] += cnt[r - 1];
        for (uint32_t i = n; i-- > 0;) tmp[--cnt[i + h < n ? rk[i + h] : 0]] = i;
        memset(cnt, 0, sizeof(uint32_t) * (m + 1));
        for (uint32_t i = 0; i < n; ++i) cnt[rk[i]]++;
        for (uint32_t r = 1; r <= m; ++r) cnt[r] += cnt[r - 1];
        for (uint32_t j = n; j-- > 0;) sa[--cnt[rk[tmp[j]]]] = tmp[j];
        uint32_t r = 1;
        nrk[sa[0]] = 1;
        for (uint32_t j = 1; j < n; ++j) {
            uint32_t a = sa[j - 1], b = sa[j];
            uint32_t a2 = a + h < n ? rk[a + h] : 0, b2 = b + h < n ? rk[b + h] : 0;
            if (rk[a] != rk[b] || a2 != b2) ++r;
            nrk[b] = r;
        }
        uint32_t* x = rk; rk = nrk; nrk = x;
        m = r;
        if (r == n) break;
    }
    free(tmp); free(rk); free(nrk); free(cnt);
    return sa;
}

void sl_free(sl_t* s) {
    if (!s) return;
    for (int l = 0; l < LEVELS; ++l) { free(s->lv[l].bits); free(s->lv[l].cum); }
    free(s->samples); free(s->text_start); free(s->text_group);
    free(s);
}

/* Builds the stand-in index. given_sa (may be NULL): the suffix array of the same text computed elsewhere — a suffix
 * array is unique, so it only saves the O(n log n) doubling here (bench.py's config-5 CPU baseline, where the build
 * is not timed); NULL sorts with build_sa. tests/test_seqan_like.py checks both give the same structure. */
sl_t* sl_build_sa(const char* seq, const uint64_t* rec_off, uint32_t n_records, const int32_t* group_of_rec,
                  uint32_t n_groups, const uint32_t* given_sa) {
    if (n_records == 0) return NULL;
    uint64_t total = 1;
    for (uint32_t r = 0; r < n_records; ++r) total += 2 * (rec_off[r + 1] - rec_off[r] + 1);
    if (total >= 0xFFFFFFF0ull) return NULL;
    const uint32_t n = (uint32_t)total;
    sl_t* s = (sl_t*)calloc(1, sizeof(sl_t));
    s->n = n; s->n_texts = 2 * n_records; s->n_groups = n_groups;
    uint8_t* t = (uint8_t*)malloc(n);
    s->text_start = (uint32_t*)malloc(sizeof(uint32_t) * (s->n_texts + 1));
    s->text_group = (int32_t*)malloc(sizeof(int32_t) * s->n_texts);
    uint32_t p = 0;
    for (uint32_t r = 0; r < n_records; ++r) {
        uint64_t b = rec_off[r], len = rec_off[r + 1] - b;
        s->text_start[2 * r] = p;
        for (uint64_t i = 0; i < len; ++i) t[p + i] = code_of((unsigned char)seq[b + i]);
        t[p + len] = S_SEP;
        uint32_t q = p + (uint32_t)len + 1;
        s->text_start[2 * r + 1] = q;
        for (uint64_t i = 0; i < len; ++i) t[q + i] = comp_code(t[p + len - 1 - i]);
        t[q + len] = S_SEP;
        p = q + (uint32_t)len + 1;
        s->text_group[2 * r] = s->text_group[2 * r + 1] = group_of_rec[r];
    }
    s->text_start[s->n_texts] = p;
    t[p] = S_TERM;
    uint32_t* sa = NULL;
    if (given_sa) {
        sa = (uint32_t*)malloc(sizeof(uint32_t) * n);
        memcpy(sa, given_sa, sizeof(uint32_t) * n);
    } else {
        sa = build_sa(t, n);
    }
    uint8_t* bwt = (uint8_t*)malloc(n);
    uint32_t cnt[SIGMA] = {0};
    for (uint32_t i = 0; i < n; ++i) {
        bwt[i] = sa[i] ? t[sa[i] - 1] : t[n - 1];
        cnt[t[i]]++;
    }
    s->C[0] = 0;
    for (int c = 0; c < SIGMA; ++c) s->C[c + 1] = s->C[c] + cnt[c];
    s->samples = (uint32_t*)malloc(sizeof(uint32_t) * (n / SAMPLE + 1));
    for (uint32_t j = 0; j * SAMPLE < n; ++j) s->samples[j] = sa[j * SAMPLE];
    free(sa);
    free(t);
    /* wavelet matrix levels */
    uint8_t* cur = bwt;
    uint8_t* nxt = (uint8_t*)malloc(n);
    const uint32_t words = n / 64 + 1;
    for (int l = 0; l < LEVELS; ++l) {
        level_t* L = &s->lv[l];
        L->bits = (uint64_t*)calloc(words, sizeof(uint64_t));
        L->cum = (uint32_t*)malloc(sizeof(uint32_t) * (words + 1));
        uint32_t z = 0;
        for (uint32_t i = 0; i < n; ++i)
            if ((cur[i] >> (LEVELS - 1 - l)) & 1) L->bits[i >> 6] |= 1ull << (i & 63);
            else ++z;
        L->zeros = z;
        uint32_t acc = 0;
        for (uint32_t w = 0; w < words; ++w) { L->cum[w] = acc; acc += (uint32_t)__builtin_popcountll(L->bits[w]); }
        L->cum[words] = acc;
        uint32_t zi = 0, oi = z;
        for (uint32_t i = 0; i < n; ++i) {
            if ((cur[i] >> (LEVELS - 1 - l)) & 1) nxt[oi++] = cur[i];
            else nxt[zi++] = cur[i];
        }
        uint8_t* x = cur; cur = nxt; nxt = x;
    }
    free(cur); free(nxt);
    for (int c = 0; c < SIGMA; ++c) s->base[c] = wm_map(s, (uint8_t)c, 0);
    return s;
}

sl_t* sl_build(const char* seq, const uint64_t* rec_off, uint32_t n_records, const int32_t* group_of_rec,
               uint32_t n_groups) {
    return sl_build_sa(seq, rec_off, n_records, group_of_rec, n_groups, NULL);
}

/* SA[16 j] samples (tests: the given-SA build equals the own build) */
uint32_t sl_sample(const sl_t* s, uint32_t j) { return j * SAMPLE < s->n ? s->samples[j] : 0xFFFFFFFFu; }

/* Backward search of k symbols (codes); returns the SA interval [lo, hi). */
static inline void search(const sl_t* s, const uint8_t* q, uint32_t k, uint32_t* lo_out, uint32_t* hi_out) {
    uint32_t lo = 0, hi = s->n;
    for (uint32_t i = k; i-- > 0 && lo < hi;) {
        lo = lf(s, q[i], lo);
        hi = lf(s, q[i], hi);
    }
    *lo_out = lo; *hi_out = hi < lo ? lo : hi;
}

static inline uint32_t text_of(const sl_t* s, uint32_t pos) {
    uint32_t a = 0, b = s->n_texts;  /* largest t with text_start[t] <= pos */
    while (b - a > 1) {
        uint32_t m = (a + b) / 2;
        if (s->text_start[m] <= pos) a = m; else b = m;
    }
    return a;
}

static int cmp_u64(const void* x, const void* y) {
    uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
    return a < b ? -1 : a > b;
}

typedef struct { uint64_t* v; size_t cap; } hits_t;

/* The reference's per-window work: search, locate every hit, sort (text_id, pos), first-hit group rule. */
static int32_t which_hit(const sl_t* s, const uint8_t* q, uint32_t k, hits_t* h) {
    uint32_t lo, hi;
    search(s, q, k, &lo, &hi);
    uint32_t m = hi - lo;
    if (m == 0) return -1;
    if (m > h->cap) { h->cap = m * 2; h->v = (uint64_t*)realloc(h->v, sizeof(uint64_t) * h->cap); }
    for (uint32_t i = 0; i < m; ++i) {
        uint32_t pos = locate(s, lo + i);
        uint32_t tid = text_of(s, pos);
        h->v[i] = ((uint64_t)tid << 32) | (pos - s->text_start[tid]);
    }
    qsort(h->v, m, sizeof(uint64_t), cmp_u64);
    int32_t w = -1;
    for (uint32_t i = 0; i < m; ++i) {
        int32_t g = s->text_group[h->v[i] >> 32];
        if (w == -1) w = g;
        else if (w != g) { w = -2; break; }
    }
    return w;
}

/* Occurrence count of an ASCII k-mer (tests). */
int64_t sl_count(const sl_t* s, const char* kmer, uint32_t k) {
    uint8_t buf[4096];
    if (k > sizeof(buf)) return -1;
    for (uint32_t i = 0; i < k; ++i) buf[i] = code_of((unsigned char)kmer[i]);
    uint32_t lo, hi;
    search(s, buf, k, &lo, &hi);
    return (int64_t)(hi - lo);
}

/* Group label of an ASCII k-mer by the reference's rule: -1 absent, -2 several groups, else the group. */
int32_t sl_which(const sl_t* s, const char* kmer, uint32_t k) {
    uint8_t buf[4096];
    if (k > sizeof(buf)) return -3;
    for (uint32_t i = 0; i < k; ++i) buf[i] = code_of((unsigned char)kmer[i]);
    hits_t h = {NULL, 0};
    int32_t w = which_hit(s, buf, k, &h);
    free(h.v);
    return w;
}

/* Read scan; same contract as oracle_scan (kmer_oracle.c): counts u64[G+2] = {T, ambiguous, U[G]}. */
int sl_scan(const sl_t* s, const char* seq, const char* qual, const uint64_t* off, uint64_t n_reads, int paired,
            uint32_t k, uint32_t cutoff, int mode, uint64_t* counts, double* weights, int threads) {
    const uint32_t G = s->n_groups;
    if (k == 0 || (paired && (n_reads & 1))) return -1;
    double lut[42];
    for (int q = 0; q < 42; ++q) lut[q] = 1.0 - 1.0 / pow(10.0, (double)q / 10.0);
    memset(counts, 0, sizeof(uint64_t) * (G + 2));
    if (weights) memset(weights, 0, sizeof(double) * G);
    const uint64_t n_units = paired ? n_reads / 2 : n_reads;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    uint64_t T = 0, amb = 0;
#pragma omp parallel num_threads(threads) reduction(+ : T, amb)
    {
        uint64_t* U = (uint64_t*)calloc(G, sizeof(uint64_t));
        double* W = (double*)calloc(G, sizeof(double));
        size_t cap = 1 << 16;
        uint8_t* sb = (uint8_t*)malloc(cap);
        uint8_t* qb = (uint8_t*)malloc(cap);
        hits_t h = {NULL, 0};
#pragma omp for schedule(dynamic, 256)
        for (uint64_t u = 0; u < n_units; ++u) {
            int which_group = -1, is_amb = 0;
            for (int mate = 0; mate < (paired ? 2 : 1); ++mate) {
                uint64_t r = paired ? 2 * u + mate : u;
                uint64_t b = off[r], L = off[r + 1] - b;
                if (L > cap) { cap = L; sb = (uint8_t*)realloc(sb, cap); qb = (uint8_t*)realloc(qb, cap); }
                for (uint64_t i = 0; i < L; ++i) {
                    sb[i] = code_of((unsigned char)seq[b + i]);
                    int q = (int)(unsigned char)qual[b + i] - 33;
                    qb[i] = (uint8_t)(q < 0 ? 0 : (q > 41 ? 41 : q));
                }
                if (L < k) continue;
                for (uint64_t j = 0; j + k <= L; ++j) {
                    uint8_t mn = 255; int has_n = 0;  /* ranges::min + find per window, as the reference (:162) */
                    for (uint32_t i = 0; i < k; ++i) { if (qb[j + i] < mn) mn = qb[j + i]; has_n |= sb[j + i] == S_N; }
                    if (!(mn > cutoff && !has_n)) continue;
                    ++T;
                    int32_t which = which_hit(s, sb + j, k, &h);
                    if (which < 0) continue;
                    ++U[which];
                    if (mode == 1) {
                        double w = 1.0;
                        for (uint32_t i = 0; i < k; ++i) w = w / lut[qb[j + i]];
                        W[which] += w;
                    }
                    if (which_group >= 0 && which_group != which) is_amb = 1;
                    else which_group = which;
                }
            }
            if (is_amb) ++amb;
        }
#pragma omp critical
        {
            for (uint32_t g = 0; g < G; ++g) {
                counts[2 + g] += U[g];
                if (weights) weights[g] += W[g];
            }
        }
        free(U); free(W); free(sb); free(qb); free(h.v);
    }
    counts[0] = T;
    counts[1] = amb;
    return 0;
}

uint32_t sl_text_len(const sl_t* s) { return s->n; }
