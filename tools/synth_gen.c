/* Multithreaded generator of the deterministic synthetic read stream (speq_amd/synth.py).
 *
 * Bench and test infrastructure only (it makes inputs; it computes no counts). It reproduces
 * synth._make_reads_chunk byte for byte — the numpy version stays the definition and tests/test_synth_gen.py checks
 * the two against each other — but runs ~100x faster, so bench.py can stage config 3's 10 M reads in seconds.
 *
 * Streams (counter-based splitmix64, value i of stream s = mix64(s * GOLDEN + (i + 1) * GOLDEN)):
 *   2: eight draws per fragment (variant, isolate, start, strand, shorten?, short length)
 *   3: substitution-error test per base, 4: substitution choice, 5: N test, 6: low-quality test
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define GOLDEN 0x9E3779B97F4A7C15ull

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t rnd(uint64_t seed, uint64_t i) { return mix64(seed * GOLDEN + (i + 1) * GOLDEN); }
static inline double unit(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

static inline uint8_t comp(uint8_t c) {
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        default: return c;
    }
}
/* np.searchsorted(b"ACGT", c) (side left): number of ACGT codes below c */
static inline int acgt_rank(uint8_t c) { return (c > 'A') + (c > 'C') + (c > 'G') + (c > 'T'); }

/* genomes: R x Lg ASCII (row-major), R = V * I. Writes n_rec = n_reads (or 2 n_reads paired) records of read_len
 * bases each into seq/qual (row-major, n_rec x read_len; a record shortened to lens[i] < read_len keeps its first
 * lens[i] bases — the caller compacts), lens[n_rec] and var[n_rec]. Returns 0, or -1 on bad arguments. */
int synth_reads(const uint8_t* genomes, uint32_t V, uint32_t I, uint64_t Lg, uint64_t n_reads, uint32_t read_len,
                uint64_t start_index, double err_rate, double n_rate, double lowq_rate, double short_frac, int paired,
                uint32_t fragment, uint8_t* seq, uint8_t* qual, int64_t* lens, int32_t* var) {
    const uint64_t span = paired ? fragment : read_len;
    if (span > Lg || V == 0 || I == 0 || (paired && fragment < read_len)) return -1;
    /* cdf = cumsum(w) / w.sum(), w = 1..V (integer-valued doubles: exact sums, one rounding per division) */
    double cdf[4096];
    if (V > 4096) return -1;
    const double S = (double)V * (double)(V + 1) / 2.0;
    double acc = 0.0;
    for (uint32_t v = 0; v < V; ++v) {
        acc += (double)(v + 1);
        cdf[v] = acc / S;
    }
    const uint64_t nrec_per = paired ? 2 : 1;
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n_reads; ++ii) {
        const uint64_t i = (uint64_t)ii, gi = start_index + i;
        uint64_t d[8];
        for (int c = 0; c < 8; ++c) d[c] = rnd(2, gi * 8 + (uint64_t)c);
        const double u = unit(d[0]);
        uint32_t vv = 0;
        while (vv < V && cdf[vv] <= u) ++vv;  /* searchsorted(cdf, u, side="right") */
        if (vv > V - 1) vv = V - 1;
        const uint64_t iso = d[1] % I, start = d[2] % (Lg - span + 1);
        const int strand = (int)(d[3] & 1ull);
        int64_t len = read_len;
        if (short_frac > 0 && unit(d[4]) < short_frac) {
            const uint64_t m = read_len / 4 ? read_len / 4 : 1;
            len = (int64_t)(d[5] % m) + 1;
        }
        const uint8_t* g = genomes + ((uint64_t)vv * I + iso) * Lg + start;
        for (uint64_t m = 0; m < nrec_per; ++m) {
            const uint64_t rec = i * nrec_per + m;             /* row in this call's output */
            const uint64_t grec = gi * nrec_per + m;           /* row in the whole stream */
            uint8_t* s = seq + rec * read_len;
            uint8_t* q = qual + rec * read_len;
            for (uint32_t c = 0; c < read_len; ++c) {
                /* position c of the strand-adjusted fragment f (f = g or revcomp(g)); mate 2 = revcomp of f's tail */
                uint64_t fp;
                int rc_mate = 0;
                if (m == 0) fp = c;
                else {
                    fp = span - 1 - c;
                    rc_mate = 1;
                }
                uint8_t b = strand ? comp(g[span - 1 - fp]) : g[fp];
                if (rc_mate) b = comp(b);
                const uint64_t fi = grec * read_len + c;
                if (unit(rnd(3, fi)) < err_rate) {
                    const uint64_t sub = rnd(4, fi);
                    b = (uint8_t)"ACGT"[(acgt_rank(b) + 1 + (int)(sub % 3ull)) % 4];
                }
                uint8_t qq = 'I';
                if (n_rate > 0 && unit(rnd(5, fi)) < n_rate) b = 'N';
                if (lowq_rate > 0 && unit(rnd(6, fi)) < lowq_rate) qq = '+';
                s[c] = b;
                q[c] = qq;
            }
            lens[rec] = len;
            var[rec] = (int32_t)vv;
        }
    }
    return 0;
}

/* The "variable" quality profile of speq_amd/synth.py (apply_quality_profile; the numpy version is the fallback and
 * computes the same bytes): base i of a record at position pos of a record of length L gets, from r = stream `seed`
 * value i, q = 40 - 4 pos / L + (r % 7 - 3), or a dip to 12 + (r >> 40) % 18 when unit(r) < 0.02 + 0.02 pos / L;
 * rint, clipped to [2, 41], written as Phred+33. */
int synth_quality_variable(const uint64_t* offsets, uint64_t n_rec, uint64_t seed, uint8_t* qual) {
#pragma omp parallel for schedule(static)
    for (uint64_t rec = 0; rec < n_rec; ++rec) {
        const uint64_t a = offsets[rec], L = offsets[rec + 1] - a;
        for (uint64_t pos = 0; pos < L; ++pos) {
            const uint64_t i = a + pos;
            const uint64_t r = rnd(seed, i);
            const double frac = (double)pos / (double)(L ? L : 1);
            double q = 40.0 - 4.0 * frac + ((double)(r % 7ull) - 3.0);
            if (unit(r) < 0.02 + 0.02 * frac) q = 12.0 + (double)((r >> 40) % 18ull);
            q = rint(q);
            q = q < 2.0 ? 2.0 : (q > 41.0 ? 41.0 : q);
            qual[i] = (uint8_t)((int)q + 33);
        }
    }
    return 0;
}
