/*
 * kmer_oracle.c — CPU ORACLE for the SPeQ scan path. TEST INFRASTRUCTURE ONLY.
 *
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only as
 *   the checker / the timed CPU baseline — never as the product path (speq_amd/ never links or loads it).
 *
 *   PARITY UNPINNED at the SeqAn3 boundary: the reference's search arithmetic lives in SeqAn 3.0.1
 *   (fm_index + search), an empty git submodule in /root/reference (deps/seqan3), and the reference ships no
 *   golden vectors. This file restates the reference's per-window SEMANTICS with an
 *   independent algorithm (a hash map from every k-mer of the indexed texts to its group label), so it
 *   shares no code or data structure with the FM-index product path. It is cross-checked against a
 *   pure-Python substring search (tests/golden/make_golden.py) on the committed fixtures.
 *
 * Restated reference behaviour (file:line in /root/reference):
 *   texts [fwd_r, revcomp(fwd_r)] per record            src/fm_indexer.cpp:25-33
 *   text t -> group group_scaffolds[t/2]                 src/fm_scanner.cpp:74-77
 *   window filter min(Q) > cutoff && no N                src/fm_scanner.cpp:162
 *   first-hit single-group rule (which_hit)              src/fm_scanner.cpp:165-177
 *   tallies T, U[g], ambiguous (first group kept)        src/fm_scanner.cpp:164, :180, :183-190, :213
 *   Phred weight w = fold(w / (1 - 1/10^(q/10)))         src/fm_scanner.cpp:454
 *   paired: both mates share one read state               src/fm_scanner.cpp:709-729 (global), :963-995 (local)
 *   reference-uniqueness (.dat) pass                      src/fm_scanner.cpp:1503-1539
 *   EM estimator pass (global temp_acc / local qavg)      src/fm_scanner.cpp:1087-1125, :1175-1219, :1273-1311,
 *                                                         :1370-1415
 * dna5 conversion (ACGT/acgt, U->T, other->N) and phred42 clamping [0,41] follow SeqAn 3.0.1 (upstream,
 * believed).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    uint32_t k, n_groups, n_records;
    uint8_t* text;          /* texts as 'A','C','G','T','N', each followed by '$' */
    uint64_t text_len;
    uint64_t* text_start;   /* 2R + 1 */
    int32_t* text_group;    /* 2R */
    uint64_t cap;           /* hash table capacity (power of two) */
    uint64_t* slot_pos;     /* window start + 1 (0 = empty) */
    int32_t* slot_label;    /* group, or -2 when the k-mer occurs in >= 2 groups */
    int64_t* slot_first;    /* head of the k-mer's occurrence list (index into occ_*), -1 = none */
    uint32_t* occ_text;     /* text id of an occurrence */
    int64_t* occ_next;      /* next occurrence of the same k-mer */
    uint64_t n_occ;
} oracle_t;

static uint8_t dna5(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 'A';
        case 'C': case 'c': return 'C';
        case 'G': case 'g': return 'G';
        case 'T': case 't': case 'U': case 'u': return 'T';
        default: return 'N';
    }
}
static uint8_t comp(uint8_t c) {
    return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'T' ? 'A' : 'N';
}
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static uint64_t hash_kmer(const uint8_t* p, uint32_t k) {
    uint64_t h = 0x9e3779b97f4a7c15ULL;
    for (uint32_t i = 0; i < k; ++i) h = (h ^ p[i]) * 0x100000001b3ULL;
    return mix64(h);
}

/* Returns the label of the k-mer at q: -1 if absent, -2 if in >= 2 groups, else the group. */
static int32_t lookup(const oracle_t* o, const uint8_t* q) {
    uint64_t m = o->cap - 1, i = hash_kmer(q, o->k) & m;
    for (;;) {
        uint64_t p = o->slot_pos[i];
        if (!p) return -1;
        if (memcmp(o->text + (p - 1), q, o->k) == 0) return o->slot_label[i];
        i = (i + 1) & m;
    }
}

void oracle_free(oracle_t* o) {
    if (!o) return;
    free(o->text); free(o->text_start); free(o->text_group); free(o->slot_pos); free(o->slot_label);
    free(o->slot_first); free(o->occ_text); free(o->occ_next);
    free(o);
}

/* Builds the k-mer -> label map over [fwd_r, rc_r] for every record. group_of_rec[r] must be >= 0. */
oracle_t* oracle_build(const char* seq, const uint64_t* rec_off, uint32_t n_records, const int32_t* group_of_rec,
                       uint32_t n_groups, uint32_t k) {
    if (k == 0 || n_records == 0) return NULL;
    oracle_t* o = (oracle_t*)calloc(1, sizeof(oracle_t));
    o->k = k; o->n_groups = n_groups; o->n_records = n_records;
    uint64_t total = 0;
    for (uint32_t r = 0; r < n_records; ++r) total += 2 * (rec_off[r + 1] - rec_off[r] + 1);
    o->text = (uint8_t*)malloc(total + 1);
    o->text_len = total;
    o->text_start = (uint64_t*)malloc(sizeof(uint64_t) * (2 * (size_t)n_records + 1));
    o->text_group = (int32_t*)malloc(sizeof(int32_t) * 2 * (size_t)n_records);
    uint64_t p = 0, n_windows = 0;
    for (uint32_t r = 0; r < n_records; ++r) {
        uint64_t b = rec_off[r], len = rec_off[r + 1] - b;
        o->text_start[2 * r] = p;
        for (uint64_t i = 0; i < len; ++i) o->text[p + i] = dna5((unsigned char)seq[b + i]);
        o->text[p + len] = '$';
        uint64_t q = p + len + 1;
        o->text_start[2 * r + 1] = q;
        for (uint64_t i = 0; i < len; ++i) o->text[q + i] = comp(o->text[p + len - 1 - i]);
        o->text[q + len] = '$';
        p = q + len + 1;
        o->text_group[2 * r] = o->text_group[2 * r + 1] = group_of_rec[r];
        if (len >= k) n_windows += 2 * (len - k + 1);
    }
    o->text_start[2 * n_records] = p;
    uint64_t cap = 16;
    while (cap < 2 * n_windows + 16) cap <<= 1;
    o->cap = cap;
    o->slot_pos = (uint64_t*)calloc(cap, sizeof(uint64_t));
    o->slot_label = (int32_t*)malloc(sizeof(int32_t) * cap);
    for (uint64_t i = 0; i < cap; ++i) o->slot_label[i] = -3; /* unset */
    o->slot_first = (int64_t*)malloc(sizeof(int64_t) * cap);
    o->occ_text = (uint32_t*)malloc(sizeof(uint32_t) * (n_windows + 1));
    o->occ_next = (int64_t*)malloc(sizeof(int64_t) * (n_windows + 1));
    /* Insertion runs on all host threads (config 5's 200 M windows: minutes on one). A slot is claimed by a CAS on
     * slot_pos; its label is the merge of the groups of every occurrence (unset + g = g, g + g = g, g + h = -2), an
     * order-free rule, so the result does not depend on the interleaving; the occurrence lists are pushed with an
     * atomic exchange, and their order only reorders additions of the same f (oracle_em_pass), which is exact. */
    memset(o->slot_first, 0xFF, sizeof(int64_t) * cap);
    uint64_t* wbase = (uint64_t*)malloc(sizeof(uint64_t) * (2 * (size_t)n_records + 1));
    wbase[0] = 0;
    for (uint32_t t = 0; t < 2 * n_records; ++t) {
        uint64_t s = o->text_start[t], e = o->text_start[t + 1] - 1;
        wbase[t + 1] = wbase[t] + (e - s >= k ? e - s - k + 1 : 0);
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t t = 0; t < 2 * (int64_t)n_records; ++t) {
        uint64_t s = o->text_start[t], e = o->text_start[t + 1] - 1;
        if (e - s < k) continue;
        const int32_t g = o->text_group[t];
        for (uint64_t w = s; w + k <= e; ++w) {
            const uint8_t* kp = o->text + w;
            uint64_t m = cap - 1, i = hash_kmer(kp, k) & m;
            for (;;) {
                uint64_t sp = __atomic_load_n(&o->slot_pos[i], __ATOMIC_ACQUIRE);
                if (!sp) {
                    uint64_t expect = 0;
                    if (__atomic_compare_exchange_n(&o->slot_pos[i], &expect, w + 1, 0, __ATOMIC_ACQ_REL,
                                                    __ATOMIC_ACQUIRE))
                        sp = w + 1;
                    else
                        sp = expect;
                }
                if (sp == w + 1 || memcmp(o->text + (sp - 1), kp, k) == 0) {
                    int32_t cur = __atomic_load_n(&o->slot_label[i], __ATOMIC_RELAXED);
                    for (;;) {
                        int32_t nxt = cur == -3 ? g : (cur == g ? g : -2);
                        if (nxt == cur ||
                            __atomic_compare_exchange_n(&o->slot_label[i], &cur, nxt, 0, __ATOMIC_RELAXED,
                                                        __ATOMIC_RELAXED))
                            break;
                    }
                    const uint64_t x = wbase[t] + (w - s);
                    o->occ_text[x] = (uint32_t)t;
                    o->occ_next[x] = __atomic_exchange_n(&o->slot_first[i], (int64_t)x, __ATOMIC_RELAXED);
                    break;
                }
                i = (i + 1) & m;
            }
        }
    }
    o->n_occ = wbase[2 * n_records];
    free(wbase);
    return o;
}

static int64_t find_slot(const oracle_t* o, const uint8_t* q) {
    uint64_t m = o->cap - 1, i = hash_kmer(q, o->k) & m;
    for (;;) {
        uint64_t p = o->slot_pos[i];
        if (!p) return -1;
        if (memcmp(o->text + (p - 1), q, o->k) == 0) return (int64_t)i;
        i = (i + 1) & m;
    }
}

/* Label of an arbitrary ASCII k-mer (for tests). */
int32_t oracle_lookup_ascii(const oracle_t* o, const char* kmer) {
    uint8_t buf[4096];
    if (o->k > sizeof(buf)) return -3;
    for (uint32_t i = 0; i < o->k; ++i) buf[i] = dna5((unsigned char)kmer[i]);
    return lookup(o, buf);
}

/*
 * Read scan. counts: u64[G+2] = {T, ambiguous, U[0..G)}; weights: f64[G] (local mode) or NULL.
 * mode 0 = global (integer tallies), 1 = local (Phred-weighted). Records 2i, 2i+1 are mates if paired.
 * Outputs are overwritten. Returns 0, or -1 on bad arguments.
 */
int oracle_scan(const oracle_t* o, const char* seq, const char* qual, const uint64_t* off, uint64_t n_reads,
                int paired, uint32_t cutoff, int mode, uint64_t* counts, double* weights, int threads) {
    const uint32_t G = o->n_groups, k = o->k;
    if (paired && (n_reads & 1)) return -1;
    double lut[42];
    for (int q = 0; q < 42; ++q) lut[q] = 1.0 - 1.0 / pow(10.0, (double)q / 10.0);
    memset(counts, 0, sizeof(uint64_t) * (G + 2));
    if (weights) memset(weights, 0, sizeof(double) * G);
    uint64_t n_units = paired ? n_reads / 2 : n_reads;
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
        uint8_t* sb = (uint8_t*)malloc(1 << 20);
        uint8_t* qb = (uint8_t*)malloc(1 << 20);
        size_t cap = 1 << 20;
#pragma omp for schedule(dynamic, 1024)
        for (uint64_t u = 0; u < n_units; ++u) {
            int which_group = -1, is_amb = 0;
            for (int m = 0; m < (paired ? 2 : 1); ++m) {
                uint64_t r = paired ? 2 * u + m : u;
                uint64_t b = off[r], L = off[r + 1] - b;
                if (L > cap) { cap = L; sb = (uint8_t*)realloc(sb, cap); qb = (uint8_t*)realloc(qb, cap); }
                for (uint64_t i = 0; i < L; ++i) {
                    sb[i] = dna5((unsigned char)seq[b + i]);
                    int q = (int)(unsigned char)qual[b + i] - 33;
                    qb[i] = (uint8_t)(q < 0 ? 0 : (q > 41 ? 41 : q));
                }
                if (L < k) continue;
                for (uint64_t j = 0; j + k <= L; ++j) {
                    int pass = 1;
                    for (uint32_t i = 0; i < k; ++i)
                        if (qb[j + i] <= cutoff || sb[j + i] == 'N') { pass = 0; break; }
                    if (!pass) continue;
                    ++T;
                    int32_t which = lookup(o, sb + j);
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
        free(U); free(W); free(sb); free(qb);
    }
    counts[0] = T;
    counts[1] = amb;
    return 0;
}

/* Reference-uniqueness pass: every window of fwd_r and rc_r, r < n_records. Outputs overwritten. */
int oracle_ref_unique(const oracle_t* o, uint64_t* u_ref, uint64_t* tot_ref) {
    const uint32_t k = o->k;
    memset(u_ref, 0, sizeof(uint64_t) * o->n_groups);
    memset(tot_ref, 0, sizeof(uint64_t) * o->n_groups);
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t t = 0; t < 2 * (int64_t)o->n_records; ++t) {
        uint64_t s = o->text_start[t], e = o->text_start[t + 1] - 1;
        int32_t g = o->text_group[t];
        if (e - s < k) continue;
        uint64_t tot = 0, u = 0;
        for (uint64_t w = s; w + k <= e; ++w) {
            ++tot;
            if (lookup(o, o->text + w) == g) ++u;
        }
        __atomic_fetch_add(&tot_ref[g], tot, __ATOMIC_RELAXED);
        __atomic_fetch_add(&u_ref[g], u, __ATOMIC_RELAXED);
    }
    return 0;
}

/*
 * One EM estimator pass, literally as the reference runs it (single-end global src/fm_scanner.cpp:1087-1125, local
 * :1175-1219, paired :1273-1311 / :1370-1415): for every passing window, hits_per_group_int[g] += f for each
 * occurrence in a text of group g (f = 1/pp - (1 - pp) in global mode, qavg = fold(a / (1 - 10^(-b/10))) -
 * (1 - fold(a * (1 - 10^(-b/10)))) in local mode), a[i] = hits_per_group_int[i] * percent[i] / counts[i],
 * norm = sum a[i] (i in order), and if norm > 0, next[i] += a[i] / norm. Single-threaded. next is overwritten.
 */
int oracle_em_pass(const oracle_t* o, const char* seq, const char* qual, const uint64_t* off, uint64_t n_reads,
                   int paired, uint32_t cutoff, int mode, double percent_perfect, const double* percent,
                   const int32_t* group_counts, double* next) {
    const uint32_t G = o->n_groups, k = o->k;
    if (paired && (n_reads & 1)) return -1;
    memset(next, 0, sizeof(double) * G);
    double* h = (double*)malloc(sizeof(double) * G);
    double* a = (double*)malloc(sizeof(double) * G);
    size_t cap = 1 << 16;
    uint8_t* sb = (uint8_t*)malloc(cap);
    uint8_t* qb = (uint8_t*)malloc(cap);
    for (uint64_t r = 0; r < n_reads; ++r) {
        uint64_t b = off[r], L = off[r + 1] - b;
        if (L > cap) { cap = L; sb = (uint8_t*)realloc(sb, cap); qb = (uint8_t*)realloc(qb, cap); }
        for (uint64_t i = 0; i < L; ++i) {
            sb[i] = dna5((unsigned char)seq[b + i]);
            int q = (int)(unsigned char)qual[b + i] - 33;
            qb[i] = (uint8_t)(q < 0 ? 0 : (q > 41 ? 41 : q));
        }
        if (L < k) continue;
        for (uint64_t j = 0; j + k <= L; ++j) {
            int pass = 1;
            for (uint32_t i = 0; i < k; ++i)
                if (qb[j + i] <= cutoff || sb[j + i] == 'N') { pass = 0; break; }
            if (!pass) continue;
            double f;
            if (mode == 0) {
                f = 1.0 / percent_perfect - (1 - percent_perfect);
            } else {
                double x = 1.0, y = 1.0;
                for (uint32_t i = 0; i < k; ++i) x = x / (1.0 - 1.0 / pow(10.0, (double)qb[j + i] / 10.0));
                for (uint32_t i = 0; i < k; ++i) y = y * (1.0 - 1.0 / pow(10.0, (double)qb[j + i] / 10.0));
                f = x - (1.0 - y);
            }
            for (uint32_t g = 0; g < G; ++g) h[g] = 0.0;
            int64_t s = find_slot(o, sb + j);
            if (s >= 0)
                for (int64_t x = o->slot_first[s]; x >= 0; x = o->occ_next[x]) h[o->text_group[o->occ_text[x]]] += f;
            double norm = 0.0;
            for (uint32_t g = 0; g < G; ++g) {
                a[g] = h[g] * percent[g] / group_counts[g];
                norm += a[g];
            }
            if (norm > 0.0)
                for (uint32_t g = 0; g < G; ++g) next[g] += a[g] / norm;
        }
    }
    free(h); free(a); free(sb); free(qb);
    return 0;
}
