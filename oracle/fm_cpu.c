/*
 * fm_cpu.c — the BUILD'S OWN ALGORITHM on host cores (SURVEY.md §8(d) CPU baseline column (ii)).
 * BASELINE INFRASTRUCTURE ONLY: loaded by bench.py's cpu_baseline leg and tests/, never by speq_amd/.
 *
 * Same search as the HIP kernel k_scan (speq_amd/csrc/scan_kernels.hip) over the same index arrays (read from a
 * built index through speq_index_array): 2-bit packed windows, q-mer table lookup, three-/two-/one-symbol LF steps
 * with the kernel's level choice, label-run classification (no locate), per-unit ambiguity as min != max of the
 * counted groups. Global mode (integer tallies) only. Shows what the label-run algorithm does on CPU cores, beside
 * seqan_like.c (the reference's algorithm) — so the GPU/CPU comparison is also made algorithm-for-algorithm.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define BLOCK 96u

typedef struct {
    const uint32_t* occ;   /* 5 planes x nb entries of 4 u32 {count, bits0, bits1, bits2} */
    const uint32_t* occ2;  /* 16 planes or NULL */
    const uint32_t* occ3;  /* 64 planes or NULL */
    const uint32_t* runs;  /* nb entries */
    const uint16_t* run_label;
    const uint32_t* prefix[3]; /* q-mer tables for q, q-1, q-2 (u32 lo, hi pairs) or NULL */
    uint32_t q, n, nb, G;
} fmcpu_view;

static inline uint32_t rank_e(const uint32_t* e, uint32_t r) {
    uint32_t c = e[0];
    for (uint32_t w = 0; w < 3; ++w) {
        const uint32_t lo = w * 32;
        if (r >= lo + 32) c += (uint32_t)__builtin_popcount(e[1 + w]);
        else if (r > lo) c += (uint32_t)__builtin_popcount(e[1 + w] & ((1u << (r - lo)) - 1u));
    }
    return c;
}

static inline uint32_t lfp(const uint32_t* planes, uint32_t nb, uint32_t plane, uint32_t i) {
    const uint32_t b = i / BLOCK;
    return rank_e(planes + 4 * ((uint64_t)plane * nb + b), i - b * BLOCK);
}

static inline uint32_t run_of(const fmcpu_view* v, uint32_t i) { return lfp(v->runs, v->nb, 0, i) ; }

static uint8_t sym_of(unsigned char ch) {
    ch |= 0x20;
    return ch == 'a' ? 0 : ch == 'c' ? 1 : ch == 'g' ? 2 : (ch == 't' || ch == 'u') ? 3 : 4;
}

/* -1 absent, -2 several groups, else the group; P = window packed 2 bits/base, last base in the low bits */
static int search(const fmcpu_view* v, uint64_t P, uint32_t k, uint32_t q_used, const uint32_t* table) {
    uint32_t lo = 0, hi = v->n;
    int32_t s = (int32_t)k;
    if (table && k >= q_used) {
        const uint64_t code = P & ((1ull << (2 * q_used)) - 1ull);
        lo = table[2 * code];
        hi = table[2 * code + 1];
        P >>= 2 * q_used;
        s -= (int32_t)q_used;
    }
    if (v->occ3) {
        const int32_t rem = s % 3;
        if (rem == 1 && lo < hi) {
            const uint32_t c = (uint32_t)(P & 3);
            lo = lfp(v->occ, v->nb, c, lo); hi = lfp(v->occ, v->nb, c, hi);
            P >>= 2; s -= 1;
        } else if (rem == 2 && lo < hi) {
            const uint32_t pl = (uint32_t)(((P >> 2) & 3) * 4 + (P & 3));
            lo = lfp(v->occ2, v->nb, pl, lo); hi = lfp(v->occ2, v->nb, pl, hi);
            P >>= 4; s -= 2;
        }
        while (s > 0 && lo < hi) {
            const uint32_t pl = (uint32_t)(((P >> 4) & 3) * 16 + ((P >> 2) & 3) * 4 + (P & 3));
            lo = lfp(v->occ3, v->nb, pl, lo); hi = lfp(v->occ3, v->nb, pl, hi);
            P >>= 6; s -= 3;
        }
    } else if (v->occ2) {
        if ((s & 1) && lo < hi) {
            const uint32_t c = (uint32_t)(P & 3);
            lo = lfp(v->occ, v->nb, c, lo); hi = lfp(v->occ, v->nb, c, hi);
            P >>= 2; s -= 1;
        }
        while (s > 0 && lo < hi) {
            const uint32_t pl = (uint32_t)(((P >> 2) & 3) * 4 + (P & 3));
            lo = lfp(v->occ2, v->nb, pl, lo); hi = lfp(v->occ2, v->nb, pl, hi);
            P >>= 4; s -= 2;
        }
    } else {
        while (s > 0 && lo < hi) {
            const uint32_t c = (uint32_t)(P & 3);
            lo = lfp(v->occ, v->nb, c, lo); hi = lfp(v->occ, v->nb, c, hi);
            P >>= 2; s -= 1;
        }
    }
    if (lo >= hi) return -1;
    const uint32_t rl = run_of(v, lo + 1), rh = run_of(v, hi);  /* run(i) = rank of boundaries in [1, i] */
    return rl == rh ? (int)v->run_label[rl] : -2;
}

/* counts u64[G+2] = {T, ambiguous, U[G]}; k <= 32 (packed windows). Returns 0, or -1 on bad arguments. */
int fmcpu_scan(const fmcpu_view* v, const char* seq, const char* qual, const uint64_t* off, uint64_t n_reads,
               int paired, uint32_t k, uint32_t cutoff, uint64_t* counts, int threads) {
    const uint32_t G = v->G;
    if (k == 0 || k > 32 || (paired && (n_reads & 1))) return -1;
    /* q-mer level: the longest of q, q-1, q-2 leaving a multiple of the widest step (as the kernel) */
    uint32_t q_used = 0;
    const uint32_t* table = NULL;
    const uint32_t step = v->occ3 ? 3 : (v->occ2 ? 2 : 1);
    for (uint32_t lvl = 0; lvl < 3 && v->q > lvl; ++lvl) {
        const uint32_t qq = v->q - lvl;
        if (!v->prefix[lvl]) break;
        if (qq <= k && (k - qq) % step == 0) { q_used = qq; table = v->prefix[lvl]; break; }
    }
    if (!table && v->q && v->prefix[0]) { q_used = v->q; table = v->prefix[0]; }
    memset(counts, 0, sizeof(uint64_t) * (G + 2));
    const uint64_t n_units = paired ? n_reads / 2 : n_reads;
#ifdef _OPENMP
    if (threads <= 0) threads = omp_get_max_threads();
#else
    threads = 1;
#endif
    uint64_t T = 0, amb = 0;
    const uint64_t kmask = k == 32 ? ~0ull : ((1ull << (2 * k)) - 1ull);
#pragma omp parallel num_threads(threads) reduction(+ : T, amb)
    {
        uint64_t* U = (uint64_t*)calloc(G, sizeof(uint64_t));
#pragma omp for schedule(dynamic, 1024)
        for (uint64_t u = 0; u < n_units; ++u) {
            int gmin = 1 << 30, gmax = -1;
            for (int m = 0; m < (paired ? 2 : 1); ++m) {
                const uint64_t r = paired ? 2 * u + m : u;
                const uint64_t b = off[r], L = off[r + 1] - b;
                uint64_t P = 0;
                uint32_t bad_run = 0; /* bases since the last bad one */
                for (uint64_t i = 0; i < L; ++i) {
                    const uint8_t c = sym_of((unsigned char)seq[b + i]);
                    int qv = (int)(unsigned char)qual[b + i] - 33;
                    qv = qv < 0 ? 0 : (qv > 41 ? 41 : qv);
                    const int bad = c == 4 || (uint32_t)qv <= cutoff;
                    P = ((P << 2) | (c & 3)) & kmask;
                    bad_run = bad ? 0 : bad_run + 1;
                    if (i + 1 < k) continue;
                    if (bad_run < k) continue;
                    ++T;
                    const int w = search(v, P, k, q_used, table);
                    if (w < 0) continue;
                    ++U[w];
                    if (w < gmin) gmin = w;
                    if (w > gmax) gmax = w;
                }
            }
            if (gmax >= 0 && gmin != gmax) ++amb;
        }
#pragma omp critical
        for (uint32_t g = 0; g < G; ++g) counts[2 + g] += U[g];
        free(U);
    }
    counts[0] = T;
    counts[1] = amb;
    return 0;
}
